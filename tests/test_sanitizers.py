"""Host-side sanitizer runs: the native runtime built with AddressSanitizer +
UBSan and with ThreadSanitizer (`make asan`, `make tsan`; device code is not instrumented),
running the C++ unit tests (watchdog thread included) and a multi-process recovery scenario
with worker deaths.  Any sanitizer report fails the test."""
import fcntl
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.slow

REPORTS = ("ERROR: AddressSanitizer", "runtime error:", "WARNING: ThreadSanitizer")


def _build(kind):
    # two test processes (pytest -n) building the same flavour would race on its object
    # directory: one make per flavour at a time
    os.makedirs(os.path.join(ROOT, "build"), exist_ok=True)
    with open(os.path.join(ROOT, "build", ".%s.lock" % kind), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        subprocess.check_call(["make", "-j8", kind], cwd=ROOT, stdout=subprocess.DEVNULL,
                              stderr=subprocess.DEVNULL)
    return os.path.join(ROOT, "build", kind, "bin")


def _env(kind):
    env = dict(os.environ)
    env["ASAN_OPTIONS"] = "detect_leaks=0"  # the HIP runtime keeps process-lifetime caches
    env["TSAN_OPTIONS"] = "halt_on_error=0"
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    return env


def _check(out):
    for r in REPORTS:
        assert r not in out, out[out.find(r) - 200:out.find(r) + 3000]


@pytest.mark.parametrize("kind", ["asan", "tsan"])
def test_unit_tests_sanitized(kind):
    bindir = _build(kind)
    p = subprocess.run([os.path.join(bindir, "unit_tests")], env=_env(kind), cwd=ROOT,
                       capture_output=True, text=True, timeout=600)
    out = p.stdout + p.stderr
    assert p.returncode == 0, out[-3000:]
    assert "0 failed" in out
    _check(out)


@pytest.mark.parametrize("kind", ["asan", "tsan"])
def test_recovery_sanitized(kind):
    bindir = _build(kind)
    cmd = [sys.executable, "-m", "rabit_amd.launcher", "-n", "4", "--num-attempt", "4",
           os.path.join(bindir, "recover_test"), "10000", "mock=0,0,1,0", "mock=1,1,1,0",
           "mock=1,1,1,1", "rabit_reduce_ring_mincount=1", "rabit_timeout=1",
           "rabit_timeout_sec=120"]
    p = subprocess.run(cmd, env=_env(kind), cwd=ROOT, capture_output=True, text=True,
                       timeout=600)
    out = p.stdout + p.stderr
    assert p.returncode == 0, out[-3000:]
    assert out.count("PASSED") == 4, out[-3000:]
    _check(out)
