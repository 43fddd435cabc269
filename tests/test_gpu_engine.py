"""Device data plane through the engine on one MI355X (world size 1, full robust path).

Multi-GPU RCCL paths cannot run on the 1-GPU box (RCCL refuses two ranks on one GPU); their
API calls run here through a one-rank communicator (test_transports_world1), the multi-rank
control flow is covered by the CPU tests and the shared-GPU direct-transport tests, and the
driver's 8-GPU bench exercises RCCL with 8 ranks.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def rabit_dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import rabit_amd as rabit
    from rabit_amd.tracker import RabitTracker

    tracker = RabitTracker("127.0.0.1", 1, port=9300, print_fn=lambda m: None).start(1)
    rabit.init(rabit_tracker_uri="127.0.0.1", rabit_tracker_port=tracker.port, rabit_task_id=0,
               rabit_world_size=1, rabit_world1_fastpath=0)
    rabit.set_error_mode(True)
    yield rabit
    rabit.finalize()
    tracker.join(30)


def test_box_libraries_match_sources():
    """on the GPU box: the libraries the tests load were built from exactly the sources of this
    tree (source hash compiled in), for gfx950 -- printed so the run's log records it"""
    from rabit_amd import _lib

    for lib in ("standard", "base", "mock"):
        info = _lib.build_info(lib)
        print("build_info", info)
        assert info["offload_arch"] == "gfx950" and info["fresh"], info


def test_device_plane_active(rabit_dev):
    assert rabit_dev.get_device() == 0
    x = torch.ones(4, device="cuda")
    h = np.zeros(4)
    assert rabit_dev.lib().RabitIsDevicePointer(x.data_ptr()) == 1
    assert rabit_dev.lib().RabitIsDevicePointer(h.ctypes.data) == 0


@pytest.mark.parametrize("op", [0, 1, 2])
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64, torch.int32, torch.int64])
def test_device_allreduce_identity(rabit_dev, op, dtype):
    x = (torch.arange(100003, device="cuda") % 97).to(dtype)
    ref = x.clone()
    rabit_dev.allreduce(x, op)
    torch.cuda.synchronize()
    assert torch.equal(x, ref)


def test_device_bitor_kernel_path(rabit_dev):
    x = torch.randint(0, 1 << 20, (5000,), dtype=torch.int32, device="cuda")
    ref = x.clone()
    rabit_dev.allreduce(x, rabit_dev.BITOR)
    torch.cuda.synchronize()
    assert torch.equal(x, ref)


def test_device_ordering_with_torch_stream(rabit_dev):
    # work queued on torch's stream right before/after the allreduce must be ordered
    x = torch.zeros(1 << 22, device="cuda")
    for i in range(5):
        x.add_(1.0)
        rabit_dev.allreduce(x, rabit_dev.SUM)
        x.mul_(2.0)
    torch.cuda.synchronize()
    assert float(x[0]) == 62.0


def test_device_prepared_allreduce(rabit_dev):
    g = torch.randn(1 << 16, device="cuda")
    out = torch.empty_like(g)
    rabit_dev.allreduce_prepared(out, g, rabit_dev.SUM, rabit_dev.PREP_SQUARE)
    torch.cuda.synchronize()
    torch.testing.assert_close(out, g * g)


def test_device_broadcast_and_allgather(rabit_dev):
    b = torch.arange(1000, dtype=torch.float32, device="cuda")
    rabit_dev.broadcast_tensor(b, 0)
    assert torch.equal(b.cpu(), torch.arange(1000, dtype=torch.float32))
    g = rabit_dev.allgather(torch.arange(10, device="cuda", dtype=torch.int64))
    assert torch.equal(g.cpu(), torch.arange(10))


def test_device_result_log_and_checkpoint(rabit_dev):
    before = rabit_dev.stats()
    x = torch.ones(1 << 20, device="cuda")
    for _ in range(3):
        rabit_dev.allreduce(x, rabit_dev.SUM)
    mid = rabit_dev.stats()
    assert mid["device_log_bytes"] >= (1 << 22)
    rabit_dev.checkpoint({"step": 1})
    after = rabit_dev.stats()
    assert after["device_log_bytes"] == 0, "checkpoint must clear the HBM result log"
    assert after["n_allreduce"] == before["n_allreduce"] + 3


def test_bench_n1(tmp_path):
    """bench.py contract at N=1 (single JSON line)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "3",
                          "--warmup", "1", "--size-mb", "16"], capture_output=True, text=True,
                         timeout=300, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    import json

    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 1 and rec["value"] > 0


@pytest.mark.parametrize("algo,extra", [("rccl", []), ("direct", []), ("auto", []),
                                        ("auto", ["rabit_rccl_tune=1", "rabit_rccl_tune_ctas=4,16"])])
def test_transports_world1(algo, extra):
    """RCCL and direct-transport API paths on the box's one GPU (a one-rank communicator /
    group): the 8-GPU runs use the same calls with more ranks."""
    from rabit_amd.launcher import LocalJob
    job = LocalJob([sys.executable, os.path.join(ROOT, "tests", "scripts", "transport_world1.py"),
                    algo] + extra, 1, 1, capture=True, timeout=240, print_fn=lambda m: None)
    rc = job.run()
    out = "".join("".join(o) for o in job.outputs)
    assert rc == 0, out[-5000:]
    assert "TRANSPORT1 OK" in out, out[-3000:]


@pytest.mark.parametrize("lib", ["base", "standard"])
def test_allreduce_graphable(lib):
    """allreduce_graphable: an ncclAllReduce captured into a hipGraph with the step's kernels
    replays exactly (base engine); the fault-tolerant engine refuses it"""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from rabit_amd.launcher import LocalJob
    job = LocalJob([sys.executable, os.path.join(ROOT, "tests", "scripts", "graph_allreduce.py"),
                    lib], 1, 1, capture=True, timeout=240, print_fn=lambda m: None)
    rc = job.run()
    out = "".join("".join(o) for o in job.outputs)
    assert rc == 0, out[-5000:]
    assert ("GRAPHAR OK" if lib == "base" else "GRAPHAR REFUSED") in out, out[-3000:]
