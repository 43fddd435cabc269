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
