"""World > 1 HBM collectives on the GPU box: several ranks share its one GPU and talk through
the direct IPC peer-memory transport (the path 8 ranks on 8 GPUs take over xGMI), including
failure and replay of device results."""
import os
import sys

import pytest

from rabit_amd.launcher import LocalJob

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(script, nworker, args=(), attempts=1, timeout=300, env=None):
    job = LocalJob([sys.executable, os.path.join(ROOT, "tests", "scripts", script)] + list(args),
                   nworker, attempts, capture=True, timeout=timeout, print_fn=lambda m: None,
                   env=env)
    rc = job.run()
    return rc, "".join("".join(o) for o in job.outputs)


@pytest.mark.parametrize("world", [2, 3, 4])
def test_direct_collectives(world):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    rc, out = _run("device_multi.py", world)
    assert rc == 0, out[-5000:]
    assert out.count("DEVMULTI OK") == world, out[-3000:]


@pytest.mark.parametrize("world", [2, 3, 4])
def test_direct_collectives_push(world):
    """the push (remote-write) reduce-scatter variant of the two-shot allreduce"""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    rc, out = _run("device_multi.py", world, ["rabit_device_direct_mode=push"])
    assert rc == 0, out[-5000:]
    assert out.count("DEVMULTI OK") == world, out[-3000:]


@pytest.mark.parametrize("mock", [[], ["mock=1,1,0,0"], ["mock=0,2,1,0", "mock=2,1,2,0"]])
@pytest.mark.parametrize("mode", ["pull", "push"])
def test_direct_recovery(mock, mode):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    rc, out = _run("device_ft.py", 3, mock + ["rabit_device_direct_mode=" + mode], attempts=4)
    assert rc == 0, out[-5000:]
    assert out.count("DEVFT OK") == 3, out[-3000:]
    if mock:
        assert "resumed at version" in out
    if len(mock) == 2:
        # the restarted ranks replayed logged HBM results: through the device broadcast path
        import re
        replays = [int(x) for x in re.findall(r"DEVFT OK replays=(\d+)", out)]
        assert sum(replays) > 0, out[-3000:]


def test_host_buffers_via_device():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    rc, out = _run("host_via_device.py", 3)
    assert rc == 0, out[-5000:]
    assert out.count("HOSTVIADEV OK") == 3, out[-3000:]


@pytest.mark.parametrize("extra", [[], ["rabit_device_symmetric_heap=64M"]])
def test_calibration_flow(extra):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    rc, out = _run("calibrate_check.py", 3, extra)
    assert rc == 0, out[-5000:]
    assert out.count("CALIB OK") == 3, out[-3000:]


@pytest.mark.parametrize("world", [2, 3])
def test_symmetric_zero_copy(world):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    rc, out = _run("symmetric_check.py", world)
    assert rc == 0, out[-5000:]
    assert out.count("SYMMETRIC OK") == world, out[-3000:]


@pytest.mark.parametrize("sym", ["0", "1"])
def test_gradient_buckets(sym):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    rc, out = _run("buckets_check.py", 2, [sym])
    assert rc == 0, out[-5000:]
    assert out.count("BUCKETS OK") == 2, out[-3000:]


@pytest.mark.parametrize("n", [2, 4])
def test_bench_torchrun_shared_gpu(n):
    """bench.py under torch.distributed.run exactly as the driver launches the N>1 runs (ranks
    share the box's GPU here, so the direct transport carries the data): the result check
    passes and rank 0 prints one JSON line."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import json
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                          "--nproc-per-node", str(n), "--master-addr", "127.0.0.1",
                          "--master-port", str(port), os.path.join(ROOT, "bench.py"),
                          "--gpus", str(n), "--steps", "3", "--warmup", "1", "--extras", "0"],
                         capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-4000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == n and rec["value"] > 0
    assert rec["transport"]["direct"] == 1, rec


@pytest.mark.parametrize("mode", ["pull", "push"])
def test_direct_half_precision(mode):
    """bf16 / fp16 allreduce (sum, max, min, fused averaging) on HBM through the direct
    transport: fp32 accumulation over all ranks, one rounding, bit-exact against torch"""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    rc, out = _run("device_half.py", 3, ["rabit_device_direct_mode=" + mode])
    assert rc == 0, out[-5000:]
    assert out.count("HALF OK") == 3, out[-3000:]

