"""Model families over several CPU ranks, with and without injected failures."""
import os
import re
import sys

import pytest

from rabit_amd.launcher import LocalJob

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCRIPT = os.path.join(ROOT, "tests", "scripts", "models_check.py")


def _run(which, n, extra=(), attempts=1):
    job = LocalJob([sys.executable, SCRIPT, which] + list(extra), n, attempts, capture=True,
                   timeout=300, print_fn=lambda m: None)
    rc = job.run()
    out = "".join("".join(o) for o in job.outputs)
    return rc, job, out


@pytest.mark.parametrize("which", ["kmeans", "linear", "gbdt"])
@pytest.mark.parametrize("n", [1, 3])
def test_model_trains(native_build, which, n):
    rc, _, out = _run(which, n)
    assert rc == 0, out[-3000:]
    assert out.count("MODEL OK") == n


@pytest.mark.parametrize("which,mock", [("kmeans", ["mock=1,3,1,0", "mock=2,5,0,0"]),
                                        ("gbdt", ["mock=2,2,3,0"]),
                                        ("linear", ["mock=0,4,2,0"])])
def test_model_survives_failures(native_build, which, mock):
    rc, job, out = _run(which, 3, mock, attempts=4)
    assert rc == 0, out[-3000:]
    assert out.count("MODEL OK") == 3
    assert sum(a - 1 for a in job.attempts) >= 1, "kill point not reached"


OVERLAP = os.path.join(ROOT, "tests", "scripts", "overlap_check.py")


def _overlap_job(mode, where, extra=(), n=3, attempts=1):
    job = LocalJob([sys.executable, OVERLAP, mode, "12", where] + list(extra), n, attempts,
                   capture=True, timeout=240, print_fn=lambda m: None)
    rc = job.run()
    out = "".join("".join(o) for o in job.outputs)
    assert rc == 0, out[-4000:]
    digests = set(re.findall(r"OVERLAP OK mode=\w+ weights=([0-9a-f]+)", out))
    assert len(digests) == 1 and out.count("OVERLAP OK") == n, out[-3000:]
    return digests.pop(), job


def test_overlapped_buckets_match_sequential(native_build):
    """CommThread + OverlappedBuckets (allreduces started from backward hooks on the comm
    thread) train to the same weights as reducing after backward, also with workers killed."""
    seq, _ = _overlap_job("seq", "cpu")
    ovl, _ = _overlap_job("overlap", "cpu")
    assert ovl == seq
    failed, job = _overlap_job("overlap", "cpu", ["lib=mock", "mock=1,1,2,0", "mock=2,2,0,0"],
                               attempts=3)
    assert sum(a - 1 for a in job.attempts) == 2, job.attempts
    assert failed == seq
