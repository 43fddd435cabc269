"""Chaos test of the host recovery path: 10 CPU workers, seeded random kill points, including
ranks that die while they serve another rank's recovery (mock_die_serving: holder or relay of a
replayed result, of a checkpoint load, of ring-replicated local state or of the bootstrap cache).

The reference exercises this path only when a second failure happens to coincide with a replay
(`/root/reference/src/allreduce_robust.cc:861-973, 1037-1088, 1103-1140`; `test/test.mk:15-37`).
Each seed: recover_test (tests/cpp/recover_test.cc) in one of its three checkpoint modes; every
rank must print PASSED (models checked against closed forms), unless the engine stopped with
"Too many nodes went down".  The seed list is fixed (SEEDS) so a failure reproduces.
"""
import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from chaos_points import draw  # noqa: E402

from rabit_amd.launcher import LocalJob  # noqa: E402

WORLD = int(os.environ.get("XRABIT_CHAOS_WORLD", "10"))  # (fuzzing other worlds)
NITER = 3
NOPS = 11  # recover_test per iteration at 10 ranks: Max, 4 string broadcasts (2 ops each), Sum, Allgather
# 32 committed seeds; XRABIT_CHAOS_SEEDS="a-b" (or "a,b,...") runs others (fuzzing)
_SPEC = os.environ.get("XRABIT_CHAOS_SEEDS", "")
SEEDS = (list(range(int(_SPEC.split("-")[0]), int(_SPEC.split("-")[1]) + 1)) if "-" in _SPEC else
         [int(s) for s in _SPEC.split(",")] if _SPEC else list(range(101, 133)))
MODES = ["global", "local", "lazy"]


def scenario(seed):
    mode = MODES[seed % 3]
    args = ["mode=" + mode, "niter=%d" % NITER, "rabit_timeout=1", "rabit_timeout_sec=60"]
    if seed % 4 == 1 and mode != "local":
        args.append("rabit_bootstrap_cache=1")
    if seed % 5 == 2:
        args.append("rabit_reduce_ring_mincount=1")  # ring allreduce
    return args + draw(seed, WORLD, NITER, NOPS)


@pytest.mark.parametrize("seed", SEEDS)
def test_host_chaos(native_build, seed):
    args = scenario(seed)
    job = LocalJob([os.path.join(native_build, "recover_test"), "200"] + args, WORLD, 10,
                   capture=True, timeout=180, print_fn=lambda m: None)
    rc = job.run()
    out = "".join("".join(o) for o in job.outputs)
    if "Too many nodes went down" in out:
        return  # every holder of some data died: the engine says so instead of hanging
    assert rc == 0, "seed %d args %s\n%s" % (seed, args, out[-4000:])
    assert out.count("PASSED") == WORLD, "seed %d args %s\n%s" % (seed, args, out[-4000:])


@pytest.mark.parametrize("where", [1, 2])
def test_chaos_hits_serving_deaths(native_build, where):
    """the serving kill points fire: rank 1 dies at op 3 of version 1, and ranks that serve its
    recovery die in turn (survivors may be blocked at op 3 or 4: a tree broadcast can complete
    on some ranks without rank 1); where=1 after the routing decision (every non-requester
    routes), where=2 once the first bytes of a transfer left (the ranks on the route)"""
    ranks = (4, 5) if where == 1 else (0, 2, 3, 4, 5)
    serving = ["mock_die_serving=%d,1,%d,0,%d" % (r, s, where) for r in ranks for s in (3, 4)]
    args = ["mode=global", "niter=3", "mock=1,1,3,0", "rabit_global_replica=10"] + serving
    job = LocalJob([os.path.join(native_build, "recover_test"), "20000"] + args, WORLD, 10,
                   capture=True, timeout=180, print_fn=lambda m: None)
    rc = job.run()
    out = "".join("".join(o) for o in job.outputs)
    assert "Hit Mock Die Serving" in out, out[-4000:]
    if "Too many nodes went down" not in out:
        assert rc == 0 and out.count("PASSED") == WORLD, out[-4000:]
