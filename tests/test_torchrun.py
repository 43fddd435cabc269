"""The torchrun launch path used by bench.py (tracker hosted by rank 0), on CPU ranks."""
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("n", [2, 4])
def test_torchrun_rendezvous(native_build, n):
    port = _free_port()
    env = dict(os.environ, rabit_device_plane="0")
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                          "--nproc-per-node", str(n), "--master-addr", "127.0.0.1",
                          "--master-port", str(port),
                          os.path.join(ROOT, "tests", "scripts", "torchrun_check.py")],
                         capture_output=True, text=True, timeout=240, cwd=ROOT, env=env)
    if out.returncode != 0:
        # the worker's own error lines first (torch.elastic's summary buries them)
        keep = [l for l in (out.stdout + out.stderr).splitlines()
                if "rabit" in l.lower() or "Error" in l or "error" in l][:40]
        raise AssertionError("\n".join(keep) + "\n----\n" + out.stderr[-3000:])
    assert out.stdout.count("TORCHRUN OK") == n


def test_torchrun_extra_params(native_build):
    """XRABIT_PARAMS reaches every rank's engine (here: consensus elision turned off)"""
    import re
    port = _free_port()
    out = {}
    for params in ("", "rabit_elide_consensus=0"):
        env = dict(os.environ, rabit_device_plane="0", XRABIT_PARAMS=params)
        r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                            "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
                            "--master-port", str(port),
                            os.path.join(ROOT, "tests", "scripts", "torchrun_check.py")],
                           capture_output=True, text=True, timeout=240, cwd=ROOT, env=env)
        assert r.returncode == 0, r.stderr[-3000:]
        out[params] = [int(x) for x in re.findall(r"elided=(\d+)", r.stdout)]
        port = _free_port()
    assert len(out[""]) == 2 and min(out[""]) > 0, out
    assert out["rabit_elide_consensus=0"] == [0, 0], out
