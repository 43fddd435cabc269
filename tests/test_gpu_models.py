"""Model families with HBM shards on the GPU box: 3 ranks share its GPU and reduce through the
direct IPC transport, with and without injected worker deaths (HBM results replayed)."""
import os
import sys

import pytest

from rabit_amd.launcher import LocalJob

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCRIPT = os.path.join(ROOT, "tests", "scripts", "models_check.py")


def _run(which, extra=(), attempts=1):
    job = LocalJob([sys.executable, SCRIPT, which, "rabit_device=0"] + list(extra), 3, attempts,
                   capture=True, timeout=300, print_fn=lambda m: None)
    rc = job.run()
    return rc, job, "".join("".join(o) for o in job.outputs)


@pytest.mark.parametrize("which,mock", [("kmeans", []), ("linear", []), ("gbdt", []),
                                        ("kmeans", ["mock=1,3,1,0"]), ("gbdt", ["mock=2,2,3,0"])])
def test_models_on_device(native_build, which, mock):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    rc, job, out = _run(which, mock, attempts=3 if mock else 1)
    assert rc == 0, out[-4000:]
    assert out.count("MODEL OK") == 3, out[-3000:]
    if mock:
        assert sum(a - 1 for a in job.attempts) >= 1, "kill point not reached"


def test_dp_train_on_hbm_with_failures(native_build):
    """examples/dp_train.py with HBM gradient buckets (fused average-allreduce over the direct
    transport, 3 ranks on the box's GPU) and device checkpoints: two workers die mid-training,
    resume from HBM snapshots and replay logged HBM results; the weights match the clean run."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from test_examples import run_dp_train
    args = ["--hidden", "4096", "--bucket-mb", "1"]
    clean, _, out0 = run_dp_train(3, 1, args)
    failed, job, out = run_dp_train(3, 3, args + ["mock=1,2,1,0", "mock=2,3,0,0"])
    assert sum(a - 1 for a in job.attempts) >= 2, "kill points did not fire"
    assert failed == clean, (clean, failed)
    import re
    assert sum(int(x) for x in re.findall(r"device_ops=(\d+)", out0)) > 0, out0[-2000:]
    assert sum(int(x) for x in re.findall(r"replays=(\d+)", out)) > 0, out[-3000:]


def test_dp_train_graphed_step_matches_eager(native_build):
    """GraphedStep: forward+backward replayed as one hipGraph, the bucket allreduce (3 ranks on
    the direct transport) outside it: the final weights equal the eager run's bit for bit, also
    with two workers killed and restarted mid-training (restarted workers capture their own
    graph).  graph_safe_linear keeps torch's column reduction out of the graph (profiles/r1_graphs)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from test_examples import run_dp_train
    args = ["--hidden", "256", "--layers", "6", "--bucket-mb", "1", "--safe-linear", "1"]
    eager, _, _ = run_dp_train(3, 1, args)
    graphed, _, out = run_dp_train(3, 1, args + ["--graph", "1"])
    assert out.count("graphed=1") == 3, out[-3000:]
    assert graphed == eager, (eager, graphed)
    failed, job, out = run_dp_train(3, 3, args + ["--graph", "1", "mock=1,2,1,0",
                                                  "mock=2,3,0,0"])
    assert sum(a - 1 for a in job.attempts) >= 2, "kill points did not fire"
    assert failed == eager, (eager, failed)


def test_graphed_step_replays_exactly():
    """GraphedStep on its own: a small MLP step (functional gradients) replayed 8 times gives
    the eager gradients every time."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from rabit_amd.parallel import GraphedStep
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(64, 256), torch.nn.Tanh(),
                                torch.nn.Linear(256, 1)).to(dev)
    params = list(model.parameters())
    x = torch.randn(128, 64, device=dev)
    y = torch.randn(128, 1, device=dev)
    grads = [torch.zeros_like(p) for p in params]

    def compute():
        loss = torch.nn.functional.mse_loss(model(x), y)
        torch._foreach_copy_(grads, list(torch.autograd.grad(loss, params)))
        return loss

    compute()
    ref = [g.clone() for g in grads]
    step = GraphedStep(compute)
    for _ in range(12):
        step()
        torch.cuda.synchronize()
        assert all(torch.equal(a, b) for a, b in zip(grads, ref))
    assert step.captured


def test_overlapped_buckets_on_device(native_build):
    """OverlappedBuckets on HBM (3 ranks on the box's GPU, direct transport): bucket
    allreduces run on the comm thread's HIP stream during backward; the weights equal those
    of reducing after backward, also with a worker killed and restarted."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import re
    script = os.path.join(ROOT, "tests", "scripts", "overlap_check.py")

    def run(mode, extra=(), attempts=1):
        job = LocalJob([sys.executable, script, mode, "10", "gpu"] + list(extra), 3, attempts,
                       capture=True, timeout=240, print_fn=lambda m: None)
        rc = job.run()
        out = "".join("".join(o) for o in job.outputs)
        assert rc == 0, out[-4000:]
        d = set(re.findall(r"weights=([0-9a-f]+)", out))
        assert len(d) == 1 and out.count("OVERLAP OK") == 3, out[-3000:]
        return d.pop(), job

    seq, _ = run("seq")
    ovl, _ = run("overlap")
    assert ovl == seq
    failed, job = run("overlap", ["lib=mock", "mock=1,1,3,0"], attempts=3)
    assert sum(a - 1 for a in job.attempts) == 1, job.attempts
    assert failed == seq
