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
