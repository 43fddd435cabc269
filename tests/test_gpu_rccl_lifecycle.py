"""RCCL communicator lifecycle under failure, on one MI355X (VERDICT r2 "next" #1).

* rccl_lifecycle_test (C++, tests/cpp/rccl_lifecycle_test.cc): a 2-rank communicator whose
  second rank never joins ends in kTimeout at the init deadline (ncclCommAbort returns), a
  probe-reported peer failure ends it in kAborted at once, and an RCCL enqueue error becomes
  kAborted with the communicator dropped; after each, a new communicator works.
* rccl_mock_recover.py: inside the robust engine an injected RCCL enqueue error is recovered
  (re-link, new device epoch, op retried) and every result is still exact.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_comm_init_abort_and_enqueue_error(native_build):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    out = subprocess.run([os.path.join(native_build, "rccl_lifecycle_test")], cwd=ROOT,
                         capture_output=True, text=True, timeout=150)
    print(out.stdout)
    print(out.stderr[-3000:])
    assert out.returncode == 0, out.stdout + out.stderr[-3000:]
    assert "rccl_lifecycle_test: OK" in out.stdout


@pytest.mark.parametrize("fail_at", [1, 4])
def test_robust_engine_recovers_rccl_error(fail_at):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    env = dict(os.environ, PYTHONPATH=ROOT)
    out = subprocess.run([sys.executable, "tests/scripts/rccl_mock_recover.py", str(fail_at)],
                         cwd=ROOT, capture_output=True, text=True, timeout=150, env=env)
    print(out.stdout)
    print(out.stderr[-3000:])
    assert out.returncode == 0, out.stderr[-3000:]
    rec = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][-1])
    assert rec["ok"]
    assert rec["rccl_aborts"] == 1
    assert rec["n_recover_events"] >= 1
    assert rec["device_epoch"] >= 2  # a new communicator after the failure
