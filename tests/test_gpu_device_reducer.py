"""rabit::DeviceReducer (user struct reductions compiled as gfx950 kernels): world 1, and
several ranks sharing the GPU through the direct transport, with a worker killed mid-way."""
import os
import subprocess

import pytest

from rabit_amd.launcher import LocalJob

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _prog(native_build):
    return os.path.join(native_build, "device_reducer_test")


def test_device_reducer_world1(native_build):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    p = subprocess.run([_prog(native_build), "70001", "rabit_world1_fastpath=0"],
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "DEVREDUCER OK" in p.stdout


@pytest.mark.parametrize("mock", [[], ["mock=1,0,1,0"]])
def test_device_reducer_multirank(native_build, mock):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    job = LocalJob([_prog(native_build), "300007", "rabit_device=0",
                    "rabit_device_peer_buffer=1M"] + mock, 3, 3, capture=True, timeout=240,
                   print_fn=lambda m: None)
    rc = job.run()
    out = "".join("".join(o) for o in job.outputs)
    assert rc == 0, out[-4000:]
    assert out.count("DEVREDUCER OK") == 3, out[-3000:]
