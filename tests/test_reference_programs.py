"""The reference's OWN test programs, unchanged, on xrabit.

The C++ programs are the reference's `test/model_recover.cc`, `local_recover.cc`,
`lazy_recover.cc` and `guide/*.cc`. They are compiled from the read-only reference tree against
xrabit's headers (`csrc/include/rabit`) and linked with `librabit_mock`. They then run the
reference's `test/test.mk` failure matrix: 10 workers, up to 20 attempts, the same `mock=` kill
points and parameters. The launcher and tracker are xrabit's.

The reference's Python scripts (`test/local_recover.py`, `guide/*.py`) run through
`python/rabit.py`, the drop-in binding module.

This is API/ABI-level parity: a reference user's code builds and passes its own checks on xrabit.
The tests skip when the reference tree is not mounted. It is mounted in the build container; on
the GPU box it is not.
"""
import os
import subprocess
import sys

import pytest

from rabit_amd.launcher import LocalJob

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.environ.get("RABIT_REFERENCE", "/root/reference")
OUT = os.path.join(ROOT, "build", "refapi")

pytestmark = pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "test")),
                                reason="reference tree not mounted")

# test/test.mk:15-37 (dmlc-submit --num-workers=10 --local-num-attempt=20 <prog> 10000 ...)
DIE = ["mock=0,0,1,0", "mock=1,1,1,0"]
SAME = DIE + ["mock=0,1,1,0", "mock=4,1,1,0", "mock=9,1,1,0"]
HARD = DIE + ["mock=1,1,1,1", "mock=0,1,1,0", "mock=4,1,1,0", "mock=9,1,1,0", "mock=8,1,2,0",
              "mock=4,1,3,0"]
TEST_MK = {
    "model_recover_10_10k": ("model_recover", DIE + [
        "rabit_bootstrap_cache=true", "rabit_debug=true", "rabit_reduce_ring_mincount=1",
        "rabit_timeout=true", "rabit_timeout_sec=5"], 2),
    "model_recover_10_10k_die_same": ("model_recover", SAME + ["rabit_bootstrap_cache=1"], 3),
    "model_recover_10_10k_die_hard": ("model_recover", HARD + ["rabit_bootstrap_cache=1"], 4),
    "local_recover_10_10k": ("local_recover", SAME + ["mock=1,1,1,1"], 3),
    "lazy_recover_10_10k_die_hard": ("lazy_recover", HARD, 4),
    "lazy_recover_10_10k_die_same": ("lazy_recover", SAME, 3),
    "ringallreduce_10_10k": ("model_recover", ["rabit_reduce_ring_mincount=10"], 0),
}

_compiled = {}


def _compile(native_build, src):
    """compile a reference source file against xrabit (once per session)"""
    name = os.path.splitext(os.path.basename(src))[0]
    if name not in _compiled:
        os.makedirs(OUT, exist_ok=True)
        # one binary per test process (xdist workers compile concurrently)
        exe = os.path.join(OUT, "%s.%d" % (name, os.getpid()))
        lib = os.path.join(ROOT, "rabit_amd", "lib")
        cmd = ["g++", "-O2", "-std=c++17", "-D__HIP_PLATFORM_AMD__",
               "-I" + os.path.join(ROOT, "csrc", "include"), "-I/opt/rocm/include", src,
               "-o", exe, "-L" + lib, "-lrabit_mock", "-Wl,-rpath," + lib]
        p = subprocess.run(cmd, capture_output=True, text=True)
        assert p.returncode == 0, "reference program %s does not build on xrabit:\n%s" % (
            src, p.stderr[-3000:])
        _compiled[name] = exe
    return _compiled[name]


def _job(cmd, n, attempts, timeout=240, env=None, cwd=None):
    job = LocalJob(cmd, n, attempts, capture=True, timeout=timeout, print_fn=lambda m: None,
                   env=env)
    rc = job.run()
    return rc, job, "".join("".join(o) for o in job.outputs)


@pytest.mark.parametrize("scenario", sorted(TEST_MK))
def test_reference_test_mk(native_build, scenario):
    prog, args, min_restarts = TEST_MK[scenario]
    exe = _compile(native_build, os.path.join(REF, "test", prog + ".cc"))
    rc, job, out = _job([exe, "10000"] + args, 10, 20)
    assert rc == 0, out[-4000:]
    assert sum(a - 1 for a in job.attempts) >= min_restarts, "kill points did not fire"


@pytest.mark.parametrize("prog", ["basic", "broadcast", "lazy_allreduce"])
def test_reference_guide_cpp(native_build, prog):
    exe = _compile(native_build, os.path.join(REF, "guide", prog + ".cc"))
    rc, job, out = _job([exe], 3, 1, timeout=60)
    assert rc == 0, out[-3000:]


def test_reference_guide_basic_output(native_build):
    """doc/guide.md:54-59: Max then Sum over a[i] = rank + i on 3 workers"""
    exe = _compile(native_build, os.path.join(REF, "guide", "basic.cc"))
    rc, job, out = _job([exe], 3, 1, timeout=60)
    assert rc == 0, out[-3000:]
    assert "after-allreduce-max: a={2, 3, 4}" in out, out[-3000:]
    assert "after-allreduce-sum: a={6, 9, 12}" in out, out[-3000:]


@pytest.mark.parametrize("script", ["test/local_recover.py", "guide/basic.py",
                                    "guide/broadcast.py", "guide/lazy_allreduce.py"])
def test_reference_python_scripts(native_build, script):
    # the scripts do sys.path.append('../python') relative to the working directory: run them
    # from tests/, so ../python is xrabit's drop-in python/rabit.py
    env = dict(os.environ, PYTHONPATH=os.pathsep.join([os.path.join(ROOT, "python"), ROOT]))
    n = 10 if "local_recover" in script else 3
    prev = os.getcwd()
    os.chdir(os.path.join(ROOT, "tests"))
    try:
        rc, job, out = _job([sys.executable, os.path.join(REF, script), "10000"], n, 1,
                            timeout=120, env=env)
    finally:
        os.chdir(prev)
    assert rc == 0, out[-3000:]
    if "local_recover" in script:
        assert out.count("iter=2") == n, out[-3000:]
