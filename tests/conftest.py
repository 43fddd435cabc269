import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: long multi-process fault-tolerance scenario")


_built = False


def ensure_built():
    """Build the native libraries and test programs once per session (no-op when current)."""
    global _built
    if not _built:
        jobs = str(min(8, os.cpu_count() or 8))
        subprocess.check_call(["make", "-j" + jobs, "libs", "tests"], cwd=ROOT,
                              stdout=subprocess.DEVNULL)
        _built = True


@pytest.fixture(scope="session")
def native_build():
    ensure_built()
    return os.path.join(ROOT, "build", "bin")


@pytest.fixture(autouse=True)
def _heartbeat(request):
    """A GPU test that runs longer than a minute says so once a minute (on stderr): a long
    multi-rank job keeps reporting which test it is in, and a hang names itself long before its
    own timeout (the job's, or pytest's --timeout) ends it with the ranks' output."""
    if request.node.get_closest_marker("gpu") is None:
        yield
        return
    import threading
    import time

    done = threading.Event()
    t0 = time.time()

    def beat():
        while not done.wait(60.0):
            sys.stderr.write("\n[heartbeat] %s running for %.0f s\n"
                             % (request.node.nodeid, time.time() - t0))
            sys.stderr.flush()

    th = threading.Thread(target=beat, daemon=True)
    th.start()
    try:
        yield
    finally:
        done.set()
        th.join(timeout=1.0)


@pytest.fixture(scope="session")
def gpu_available():
    import torch

    return torch.cuda.is_available()
