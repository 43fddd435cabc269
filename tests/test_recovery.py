"""Multi-process fault-tolerance scenarios on CPU ranks (the reference's test/test.mk matrix).

Each scenario launches 10 worker processes through rabit_amd.launcher (tracker + restarts).
`mock=rank,version,seqno,trial` kill points make workers die; the launcher restarts them and
they recover their checkpoint and replay missed collective results from the survivors.
"""
import os
import sys

import pytest

from rabit_amd.launcher import LocalJob

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

DIE = ["mock=0,0,1,0", "mock=1,1,1,0"]
DIE_SAME = DIE + ["mock=0,1,1,0", "mock=4,1,1,0", "mock=9,1,1,0"]
DIE_HARD = DIE + ["mock=1,1,1,1", "mock=0,1,1,0", "mock=4,1,1,0", "mock=9,1,1,0",
                  "mock=8,1,2,0", "mock=4,1,3,0"]
LOCAL = DIE_SAME + ["mock=1,1,1,1"]

SCENARIOS = {
    # name: (extra args, expected restarts >= )
    "model_recover_die": (["mode=global", "rabit_bootstrap_cache=true", "rabit_debug=true",
                           "rabit_reduce_ring_mincount=1", "rabit_timeout=true",
                           "rabit_timeout_sec=20"] + DIE, 2),
    "model_recover_die_same": (["mode=global", "rabit_bootstrap_cache=1"] + DIE_SAME, 3),
    "model_recover_die_hard": (["mode=global", "rabit_bootstrap_cache=1"] + DIE_HARD, 4),
    "model_recover_die_hard_elided": (["mode=global"] + DIE_HARD, 4),
    "model_recover_die_hard_no_elide": (["mode=global", "rabit_elide_consensus=0"] + DIE_HARD, 4),
    "local_recover": (["mode=local"] + LOCAL, 3),
    "local_recover_force_local": (["mode=local", "force_local=1"] + LOCAL, 3),
    "lazy_recover_die_hard": (["mode=lazy"] + DIE_HARD, 4),
    "lazy_recover_die_same": (["mode=lazy"] + DIE_SAME, 3),
    # a death in op 0 of a version with the bootstrap cache on: the survivors' seqno (0)
    # equals the restarted rank's bootstrap seqno (found by tests/test_chaos.py, seed 129)
    "bootstrap_cache_kill_at_op0": (["mode=global", "rabit_bootstrap_cache=1", "mock=8,1,0,0",
                                     "mock=3,2,0,0"], 2),
    "ringallreduce": (["mode=global", "rabit_reduce_ring_mincount=10"], 0),
    "tree_only_small_buffer": (["mode=global", "rabit_reduce_ring_mincount=100000",
                                "rabit_reduce_buffer=4K", "rabit_tree_reduce_minsize=1K"] + DIE, 2),
}


def _run(cmd, n=10, attempts=20, timeout=240, env=None):
    job = LocalJob(cmd, n, attempts, env=env, capture=True, timeout=timeout,
                   print_fn=lambda m: None)
    rc = job.run()
    out = "".join("".join(o) for o in job.outputs)
    return rc, job, out


@pytest.mark.parametrize("name", sorted(SCENARIOS))
def test_recover_scenario(native_build, name):
    args, min_restarts = SCENARIOS[name]
    rc, job, out = _run([os.path.join(native_build, "recover_test"), "1000"] + args)
    assert rc == 0, out[-4000:]
    assert out.count("PASSED") == 10, out[-4000:]
    restarts = sum(a - 1 for a in job.attempts)
    assert restarts >= min_restarts, "expected kills did not happen (%d)" % restarts


def test_python_local_recover(native_build):
    """The reference's test/local_recover.py: pickled global + local models under failures."""
    script = os.path.join(ROOT, "tests", "scripts", "local_recover.py")
    rc, job, out = _run([sys.executable, script] + LOCAL, timeout=240)
    assert rc == 0, out[-4000:]
    assert out.count("DONE") == 10, out[-3000:]
    assert sum(a - 1 for a in job.attempts) >= 3


@pytest.mark.parametrize("elide", ["1", "0"])
def test_leaf_dies_during_small_broadcasts(native_build, elide):
    """Leaves die inside runs of small broadcasts while each result is kept on only half of the
    ranks (retention round 2): with consensus elision survivors may run ahead of the failure
    before a link error stops them, and every rank must still end with the exact results."""
    script = os.path.join(ROOT, "tests", "scripts", "bcast_leaf_fail.py")
    rc, job, out = _run([sys.executable, script, "rabit_global_replica=5",
                         "rabit_elide_consensus=" + elide, "mock=9,1,21,0", "mock=8,2,5,0",
                         "mock=9,2,40,1", "mock=7,3,2,0"], timeout=300)
    assert rc == 0, out[-4000:]
    assert out.count("BCAST-LEAF OK") == 10, out[-3000:]
    assert sum(a - 1 for a in job.attempts) >= 4


def test_lazy_prepare_not_rerun_on_replay(native_build):
    """A restarted worker must not call prepare_fun for results it replays."""
    script = os.path.join(ROOT, "tests", "scripts", "lazy_prepare.py")
    rc, job, out = _run([sys.executable, script, "mock=1,0,1,0"], n=4, attempts=3)
    assert rc == 0, out[-4000:]
    assert out.count("DONE") == 4
    # rank 1 died at seq 1 of version 0 and replayed seq 0 without preparing it again
    assert "[1] replayed-prepare-skipped" in out, out[-3000:]


@pytest.mark.parametrize("mode,kills", [("global", DIE_HARD), ("local", LOCAL), ("lazy", DIE_SAME)])
def test_recover_shared_memory_transport(native_build, mode, kills):
    """Large host ops take the shared-memory transport between co-located ranks; kills in the
    middle of the job force the group to be rebuilt after every recovery (and a restarted
    worker to join a new one) while the replay protocol serves the missed results."""
    args = ["mode=" + mode, "rabit_host_shm_min=64K", "rabit_host_shm_buffer=1M"] + kills
    rc, job, out = _run([os.path.join(native_build, "recover_test"), "70000"] + args, n=6)
    assert rc == 0, out[-4000:]
    assert out.count("PASSED") == 6, out[-4000:]
    assert sum(a - 1 for a in job.attempts) >= 2
    import re
    assert all(int(k) > 0 for k in re.findall(r"PASSED shm_ops=(-?\d+)", out)), out[-2000:]


def test_hang_in_prepare_becomes_a_recoverable_failure(native_build):
    """rabit_hang_timeout_sec: a rank stuck in its own prepare function (not waiting on anyone)
    exits for a restart; the job finishes with the same model as a clean run."""
    script = os.path.join(ROOT, "tests", "scripts", "hang_prepare.py")
    rc, job, out = _run([sys.executable, script, "rabit_hang_timeout_sec=2"], n=4, attempts=3,
                        timeout=180)
    assert rc == 0, out[-4000:]
    assert out.count("DONE") == 4, out[-3000:]
    assert "[2] prepare stuck" in out and "exiting for a restart" in out, out[-3000:]
    assert job.attempts[2] == 2 and sum(job.attempts) == 5, job.attempts


def test_mock_hang_detected_by_hang_timeout(native_build):
    """mock_hang= freezes a rank inside a collective; the hang timeout turns it into a restart
    and the reference's failure test passes on every rank."""
    rc, job, out = _run([os.path.join(native_build, "recover_test"), "1000", "mode=global",
                         "rabit_hang_timeout_sec=2", "mock_hang=3,1,1,0"], n=6, attempts=3,
                        timeout=180)
    assert rc == 0, out[-4000:]
    assert out.count("PASSED") == 6, out[-4000:]
    assert "Hit Mock Hang" in out and "exiting for a restart" in out, out[-3000:]
    assert job.attempts[3] == 2, job.attempts


def test_config5_robust_bench_model_check(native_build):
    """BASELINE config 5 on the host path (tools/robust_bench.py): allreduce + CheckPoint every
    iteration, rank 3 killed after checkpoint 2 and restarted; every rank, the restarted one
    included, must end with the closed-form model."""
    script = os.path.join(ROOT, "tools", "robust_bench.py")
    env = {"XR_ITERS": "5", "PYTHONPATH": ROOT}
    rc, job, out = _run([sys.executable, script, "mock=3,2,0,0"], n=4, attempts=3, env=env)
    assert rc == 0, out[-4000:]
    assert out.count('"model_check": {"ok": true') == 4, out[-4000:]
    assert job.attempts[3] == 2, job.attempts


@pytest.mark.gpu
def test_config5_robust_bench_model_check_hbm(native_build):
    """Config 5 on HBM: 4 ranks on GPU 0 (direct transport), 256 MiB device allreduce + HBM
    checkpoint every iteration, rank 3 killed and reloaded from a survivor's snapshot."""
    script = os.path.join(ROOT, "tools", "robust_bench.py")
    env = {"XR_ITERS": "6", "PYTHONPATH": ROOT}
    rc, job, out = _run([sys.executable, script, "mock=3,3,0,0"], n=4, attempts=3, env=env,
                        timeout=110)
    assert rc == 0, out[-4000:]
    assert out.count('"device": true') == 4, out[-4000:]
    assert out.count('"model_check": {"ok": true') == 4, out[-4000:]
    assert job.attempts[3] == 2, job.attempts
