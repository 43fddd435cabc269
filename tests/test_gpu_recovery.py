"""Fault tolerance with HBM state on the GPU box: several workers share its one GPU, collectives
use host arrays, model checkpoints are HBM snapshots; a restarted worker's model comes back
by device broadcasts (direct IPC transport) from a survivor's snapshot."""
import os
import sys

import pytest

from rabit_amd.launcher import LocalJob

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("mock", [[], ["mock=1,2,1,0"], ["mock=0,1,0,0", "mock=2,3,1,0"]])
def test_device_checkpoint_recovery(mock):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    script = os.path.join(ROOT, "tests", "scripts", "device_ckpt_recover.py")
    job = LocalJob([sys.executable, script] + mock, 3, 4, capture=True, timeout=240,
                   print_fn=lambda m: None)
    rc = job.run()
    out = "".join("".join(o) for o in job.outputs)
    assert rc == 0, out[-4000:]
    assert out.count("DEVCKPT OK") == 3
    if mock:
        assert "reloaded version" in out
        # the model came back by device broadcasts from a survivor's HBM snapshot
        import re
        loads = [int(x) for x in re.findall(r"device loads (\d+)", out)]
        assert loads and min(loads) >= 1, out[-3000:]


@pytest.mark.parametrize("replay", ["1", "0"])
def test_device_checkpoint_recovery_two_slots(replay):
    """the lean layout: 2 HBM snapshot slots (2x model, as the reference's old + new copy) and
    no proactive host mirror; replay=0 serves the restarted rank over TCP, so the survivor's
    shared pinned buffer is filled on demand from the acknowledged slot"""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import re
    script = os.path.join(ROOT, "tests", "scripts", "device_ckpt_recover.py")
    job = LocalJob([sys.executable, script, "mock=0,1,0,0", "mock=2,3,1,0",
                    "rabit_device_ckpt_slots=2", "rabit_device_ckpt_mirror=off",
                    "rabit_device_replay=" + replay], 3, 4, capture=True, timeout=240,
                   print_fn=lambda m: None)
    rc = job.run()
    out = "".join("".join(o) for o in job.outputs)
    assert rc == 0, out[-4000:]
    assert out.count("DEVCKPT OK") == 3, out[-3000:]
    assert "reloaded version" in out
    # (a rank restarted after the last checkpoint never snapshots again: 0 slots)
    slots = set(re.findall(r"slots=(\d+)", out))
    assert "2" in slots and slots <= {"0", "2"}, out[-3000:]
    # two slots of (64 Ki floats + 7 doubles) each, 256-byte rounded
    hbm = [int(x) for x in re.findall(r"hbm=(\d+)", out)]
    assert max(hbm) <= 2 * ((1 << 18) + 256), hbm


@pytest.mark.parametrize("engine", ["kernel", "hip", "sdma"])
def test_device_checkpoint_mirror_copy_engines(engine):
    """the pinned host mirror written by each copy engine (a narrow copy kernel of 8
    workgroups, hipMemcpyAsync, an SDMA engine driven through ROCr) is what a restarted rank
    gets over TCP (replay=0, every checkpoint mirrored): its model must come back exactly"""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import re
    script = os.path.join(ROOT, "tests", "scripts", "device_ckpt_recover.py")
    job = LocalJob([sys.executable, script, "mock=0,1,0,0", "mock=2,3,1,0",
                    "rabit_device_ckpt_mirror=always", "rabit_device_mirror_engine=" + engine,
                    "rabit_device_mirror_ctas=8", "rabit_device_mirror_priority=low",
                    "rabit_device_replay=0"], 3, 4, capture=True, timeout=240,
                   print_fn=lambda m: None)
    rc = job.run()
    out = "".join("".join(o) for o in job.outputs)
    assert rc == 0, out[-4000:]
    assert out.count("DEVCKPT OK") == 3, out[-3000:]
    assert "reloaded version" in out
    want = {"hip": "0", "kernel": "1", "sdma": "2"}[engine]
    assert set(re.findall(r"engine=(\d)", out)) == {want}, out[-3000:]
