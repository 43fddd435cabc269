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
