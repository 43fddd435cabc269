"""World > 1 HBM collectives on the GPU box: several ranks share its one GPU and talk through
the direct IPC peer-memory transport (the path 8 ranks on 8 GPUs take over xGMI), including
failure and replay of device results."""
import os
import sys

import pytest

from rabit_amd.launcher import LocalJob

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(script, nworker, args=(), attempts=1, timeout=300, env=None):
    job = LocalJob([sys.executable, os.path.join(ROOT, "tests", "scripts", script)] + list(args),
                   nworker, attempts, capture=True, timeout=timeout, print_fn=lambda m: None,
                   env=env)
    rc = job.run()
    return rc, "".join("".join(o) for o in job.outputs)


@pytest.mark.parametrize("fused", ["1", "0"])
@pytest.mark.parametrize("world", [2, 3, 4])
def test_direct_collectives(world, fused):
    """fused=1: two-shot chunks as one kernel with per-tile hand-offs and small ops as one
    one-shot kernel; 0: the 5-launch two-shot form and the 3-launch one-shot form"""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    rc, out = _run("device_multi.py", world, ["rabit_device_fused=" + fused,
                                              "rabit_device_fused_oneshot=" + fused])
    assert rc == 0, out[-5000:]
    assert out.count("DEVMULTI OK") == world, out[-3000:]


# the pipelined push form with 256 KiB chunks: the suite's 3 MiB ops take several rounds
PIPELINED = ["rabit_device_direct_mode=pipelined", "rabit_device_pipeline_chunk=256K"]


@pytest.mark.parametrize("mode", ["push", "pipelined"])
@pytest.mark.parametrize("world", [2, 3, 4])
def test_direct_collectives_push(world, mode):
    """the push (remote-write) reduce-scatter variant of the two-shot allreduce, and its
    pipelined form (the push of chunk k and the gather of chunk k-2 in one round, ar_plan.h)"""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    rc, out = _run("device_multi.py", world,
                   PIPELINED if mode == "pipelined" else ["rabit_device_direct_mode=push"])
    assert rc == 0, out[-5000:]
    assert out.count("DEVMULTI OK") == world, out[-3000:]


@pytest.mark.parametrize("fused", ["0", "1"])
@pytest.mark.parametrize("mock", [[], ["mock=1,1,0,0"], ["mock=0,2,1,0", "mock=2,1,2,0"]])
@pytest.mark.parametrize("mode", ["pull", "push", "pipelined"])
def test_direct_recovery(mock, mode, fused):
    """kills at fixed points, every form of the two-shot path (fused=1: the survivors' fused
    kernels give up on the abort word, the guard word keeps later launches of the group idle)"""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    if mode == "pipelined" and fused == "1":
        pytest.skip("the pipelined form has no fused variant")
    rc, out = _run("device_ft.py", 3, mock + ["rabit_device_direct_mode=" + mode,
                                              "rabit_device_fused=" + fused,
                                              "rabit_device_fused_oneshot=" + fused], attempts=4)
    assert rc == 0, out[-5000:]
    assert out.count("DEVFT OK") == 3, out[-3000:]
    if mock:
        assert "resumed at version" in out
    if len(mock) == 2:
        # the restarted ranks replayed logged HBM results: through the device broadcast path
        import re
        replays = [int(x) for x in re.findall(r"DEVFT OK replays=(\d+)", out)]
        assert sum(replays) > 0, out[-3000:]


@pytest.mark.parametrize("mode", ["pull", "push", "pipelined"])
def test_death_inside_multi_chunk_allreduce(mode):
    """mock_die_mid: rank 1 leaves in the middle of a multi-chunk device allreduce, after every
    peer has gathered the op's first chunk.  The survivors fail the op part-way; their user
    buffers must still hold the inputs (the chunks before the last reach the user buffer only
    through a copy guarded by the group's failure word), or the retry would sum partial results
    and the final model would miss its closed form."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    rc, out = _run("device_ft.py", 3, ["mock_die_mid=1,1,0,0", "rabit_device_direct_mode=" + mode,
                                       "rabit_device_fused=0"], attempts=3)
    assert rc == 0, out[-5000:]
    assert out.count("DEVFT OK") == 3, out[-3000:]
    assert "Hit Mock Die Mid Op" in out, out[-3000:]
    assert "resumed at version" in out, out[-3000:]


@pytest.mark.parametrize("world", [2, 3])
def test_link_probe(world):
    """rabit.link_probe(): per-link and all-link copy bandwidth over the IPC mappings (xGMI on
    separate GPUs, HBM here); the transport stays exact afterwards"""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    rc, out = _run("link_probe_check.py", world)
    assert rc == 0, out[-5000:]
    assert out.count("LINKPROBE OK") == world, out[-3000:]


@pytest.mark.parametrize("world", [2, 3])
def test_graphable_allreduce_direct_multirank(world):
    """allreduce_graphable over the direct transport captured into hipGraphs and replayed with
    several ranks: device-numbered barriers resynchronise every replay, eager ops in between
    stay exact, and a graphed data-parallel step reduces world x the local gradient"""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    rc, out = _run("graph_direct.py", world)
    assert rc == 0, out[-5000:]
    assert out.count("GRAPHDIRECT OK") == world, out[-3000:]


def test_result_log_spills_to_host():
    """an HBM result log capped below one iteration's results: the entries past the cap live in
    pinned host memory, and killed ranks replay both kinds (HBM and spilled) from survivors"""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import re
    rc, out = _run("device_ft.py", 3, ["mock=0,2,1,0", "mock=2,1,2,0", "rabit_device_log_cap=3M",
                                       "rabit_device_log_chunk=2M"], attempts=4)
    assert rc == 0, out[-5000:]
    assert out.count("DEVFT OK") == 3, out[-3000:]
    spilled = [int(x) for x in re.findall(r"DEVFT OK .* spilled=(\d+)", out)]
    spill_replays = [int(x) for x in re.findall(r"spilled_replays=(\d+)", out)]
    replays = [int(x) for x in re.findall(r"DEVFT OK replays=(\d+)", out)]
    assert min(spilled) > 0, out[-3000:]
    assert sum(spill_replays) > 0 and sum(replays) > 0, out[-3000:]


@pytest.mark.parametrize("extra", [["rabit_host_stage=0"],
                                   ["rabit_host_stage=1", "rabit_host_stage_chunk=1M",
                                    "rabit_host_stage_threads=3"],
                                   ["rabit_host_stage=auto", "rabit_host_stage_chunk=1M"]])
def test_host_buffers_via_device(extra):
    """host buffers through HBM: one whole copy each way, the pipelined stager, and the timed
    choice between them (agreed on every rank)"""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    rc, out = _run("host_via_device.py", 3, extra)
    assert rc == 0, out[-5000:]
    assert out.count("HOSTVIADEV OK") == 3, out[-3000:]


@pytest.mark.parametrize("mock", [["mock=1,2,1,0"], ["mock=1,2,1,0", "mock=2,3,0,0"]])
def test_host_stage_auto_across_restart(mock):
    """host buffers staged through HBM with rabit_host_stage=auto: a rank killed after the
    survivors settled on a staging form comes back, and every rank still runs the same
    collectives (the trial restarts on all ranks with the device epoch)"""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    rc, out = _run("host_stage_recover.py", 3, mock, attempts=4)
    assert rc == 0, out[-5000:]
    assert out.count("HOSTSTAGE RECOVER OK") == 3, out[-3000:]
    assert "resumed at version" in out, out[-3000:]


@pytest.mark.parametrize("world,args", [(2, []), (4, []), (3, ["rabit_device_allgather_resolve=0"])])
def test_allgather_layout_resolved_on_device(world, args):
    """device Allgather over the direct transport with no host round for the slice layout:
    variable, wrapping, repeated and changed slices over several stage windows, byte-exact"""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    rc, out = _run("allgather_resolved.py", world, args)
    assert rc == 0, out[-5000:]
    assert out.count("AGRESOLVED OK") == world, out[-3000:]


# seeded chaos on the device path (4 ranks sharing the GPU, tests/scripts/device_ft.py: a Sum,
# a Max and a 3-chunk broadcast per iteration, then an HBM checkpoint): 1-3 kill points per seed,
# among them deaths of ranks that serve a replay or a checkpoint load (routing, device exchange)
# (the seeds with a serving death among the first 15, plus two plain ones)
# the committed seeds; XRABIT_DEVICE_CHAOS_SEEDS="a,b,..." runs others (fuzzing on the GPU box)
DEVICE_CHAOS_SEEDS = ([int(s) for s in os.environ["XRABIT_DEVICE_CHAOS_SEEDS"].split(",")]
                      if os.environ.get("XRABIT_DEVICE_CHAOS_SEEDS") else
                      [201, 202, 204, 205, 207, 209, 211, 212, 214, 208])


@pytest.mark.parametrize("seed", DEVICE_CHAOS_SEEDS)
def test_device_chaos(seed):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from chaos_points import draw
    world = int(os.environ.get("XRABIT_DEVICE_CHAOS_WORLD", "4"))  # (fuzzing: up to 8)
    points = draw(seed, world, 4, 3, wheres=(0, 3, 3, 1))
    rc, out = _run("device_ft.py", world, points, attempts=6, timeout=240)
    if "Too many nodes went down" in out:
        return  # every holder of some data died: the engine says so instead of hanging
    assert rc == 0, "seed %d points %s\n%s" % (seed, points, out[-5000:])
    assert out.count("DEVFT OK") == world, "seed %d points %s\n%s" % (seed, points,
                                                                      out[-3000:])


def test_recovery_epoch_adopts_calibration():
    """after a kill, the next device epoch takes the survivors' calibration (one verified op per
    transport) instead of re-measuring it, on the restarted rank as on the survivors"""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    rc, out = _run("calib_adopt_check.py", 3, ["mock=1,1,0,0"], attempts=3)
    assert rc == 0, out[-5000:]
    assert out.count("CALIBADOPT OK") == 3, out[-3000:]


@pytest.mark.parametrize("extra", [[], ["rabit_device_symmetric_heap=160M"],
                                   ["rabit_device_fused=auto"]])
def test_calibration_flow(extra):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    # rabit_debug: each calibration point is logged, so a stalled run shows where it stood
    rc, out = _run("calibrate_check.py", 3, extra + ["rabit_debug=1"], timeout=170)
    assert rc == 0, out[-5000:]
    assert out.count("CALIB OK") == 3, out[-3000:]


@pytest.mark.parametrize("world", [2, 3])
def test_symmetric_zero_copy(world):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    rc, out = _run("symmetric_check.py", world)
    assert rc == 0, out[-5000:]
    assert out.count("SYMMETRIC OK") == world, out[-3000:]


@pytest.mark.parametrize("world,args", [(2, []), (4, []), (3, ["rabit_device_direct_mode=push"]),
                                         (2, ["rabit_device_zero_copy=0"])])
def test_registered_zero_copy(world, args):
    """ordinary torch allocations read in place by the peers once IPC-registered: reused,
    offset, unaligned, freed-and-reallocated and slot-evicted buffers stay bit-exact"""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    rc, out = _run("zero_copy_check.py", world, args)
    assert rc == 0, out[-5000:]
    assert out.count("ZEROCOPY OK") == world, out[-3000:]


def test_registered_zero_copy_expandable_segments():
    """torch's expandable segments are VMM allocations: inputs the registry cannot export are
    staged (the fallback the registry promises), mapped ones read in place; exact either way"""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    rc, out = _run("zero_copy_check.py", 2, [],
                   env={"PYTORCH_HIP_ALLOC_CONF": "expandable_segments:True"})
    assert rc == 0, out[-5000:]
    assert out.count("ZEROCOPY OK") == 2, out[-3000:]
    print([l for l in out.splitlines() if "ZEROCOPY OK" in l][0])


@pytest.mark.parametrize("sym", ["0", "1"])
def test_gradient_buckets(sym):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    rc, out = _run("buckets_check.py", 2, [sym])
    assert rc == 0, out[-5000:]
    assert out.count("BUCKETS OK") == 2, out[-3000:]


@pytest.mark.parametrize("n", [2, 4])
def test_bench_torchrun_shared_gpu(n):
    """bench.py under torch.distributed.run exactly as the driver launches the N>1 runs (ranks
    share the box's GPU here, so the direct transport carries the data): the result check
    passes and rank 0 prints one JSON line."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import json
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                          "--nproc-per-node", str(n), "--master-addr", "127.0.0.1",
                          "--master-port", str(port), os.path.join(ROOT, "bench.py"),
                          "--gpus", str(n), "--steps", "3", "--warmup", "1", "--extras", "0"],
                         capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-4000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == n and rec["value"] > 0
    assert rec["value"] == rec["busbw_GBps"] and rec["value_is"] == "busbw_GBps", rec
    assert rec["transport"]["direct"] == 1, rec
    assert rec["result_check"], rec
    if rec.get("extras"):
        assert all(v > 0 for v in rec["extras"]["link_probe_min_over_ranks"].values()), rec["extras"]
    assert "post_headline_failure" not in rec, rec["post_headline_failure"]
    # every available transport x input variant ran and matched the host fp64 reference
    ran = [v for v in rec["variants"] if v["available"]]
    assert {(v["transport"], v["input"]) for v in ran} >= {
        ("direct-%s-%s" % (m, f), i) for m in ("pull", "push") for f in ("classic", "fused")
        for i in ("torch", "symmetric")} | {
        ("direct-push-pipelined", i) for i in ("torch", "symmetric")}, rec["variants"]
    assert all(v["check"] and v["t_us"] > 0 for v in ran), rec["variants"]
    # where the classic direct form's time goes, per phase, for pull and push
    br = {b["transport"]: b for b in rec["direct_phase_breakdown"]}
    assert set(br) == {"direct-pull-classic", "direct-push-classic"}, br
    for b in br.values():
        assert b["timed_ops"] == 5 and set(b["phase_us"]) == {
            "stage", "barrier1", "reduce", "barrier2", "gather"}, b
        assert all(t >= 0 for t in b["phase_us"].values()) and b["phase_us"]["gather"] > 0, b


@pytest.mark.parametrize("mode", ["pull", "push", "pipelined"])
def test_direct_half_precision(mode):
    """bf16 / fp16 allreduce (sum, max, min, fused averaging) on HBM through the direct
    transport: fp32 accumulation over all ranks, one rounding, bit-exact against torch"""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    rc, out = _run("device_half.py", 3, ["rabit_device_direct_mode=" + mode])
    assert rc == 0, out[-5000:]
    assert out.count("HALF OK") == 3, out[-3000:]



# the LOCAL kill matrix of tests/test_recovery.py, scaled to 5 ranks: deaths at the checkpoint
# call (seq 1), repeated deaths of one rank, and a death inside the allreduce (seq 0)
LOCAL_KILLS = ["mock=0,0,1,0", "mock=1,1,1,0", "mock=0,1,1,0", "mock=3,1,1,0", "mock=1,1,1,1",
               "mock=2,2,0,0"]


@pytest.mark.parametrize("extra", [[], ["force_local=1"]])
def test_device_local_checkpoint_recovery(extra):
    """local tensors (per-rank state) checkpointed in HBM and replicated to the ring successors
    by device copies; restarted ranks get them back bit for bit (force_local=1: the global
    tensors travel as local state too)"""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    rc, out = _run("device_local.py", 5, LOCAL_KILLS + extra, attempts=4, timeout=300)
    assert rc == 0, out[-5000:]
    assert out.count("DEVLOCAL OK") == 5, out[-3000:]
    assert "local tensors intact" in out, out[-3000:]
    import re
    got = [int(x) for x in re.findall(r"DEVLOCAL OK bytes_local_in=(\d+)", out)]
    assert all(g > 0 for g in got), got


@pytest.mark.parametrize("fused", ["0", "1"])
@pytest.mark.parametrize("mode", ["pull", "push"])
def test_device_hang_detected_and_recovered(mode, fused):
    """mock_dev_hang: rank 1 stays alive but its GPU stream wedges right before a device
    allreduce.  The survivors' barriers give up, they abort and re-link; rank 1 finds its own
    stream still stuck after the abort and exits for a restart; the job finishes with the
    closed-form model."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    rc, out = _run("device_ft.py", 3, ["mock_dev_hang=1,1,0,0", "rabit_device_drain_timeout_sec=5",
                                       "rabit_device_direct_mode=" + mode,
                                       "rabit_device_fused=" + fused], attempts=3, timeout=240)
    assert rc == 0, out[-5000:]
    assert out.count("DEVFT OK") == 3, out[-3000:]
    assert "Hit Mock Device Hang" in out and "device stream wedged" in out, out[-3000:]
    assert "resumed at version" in out, out[-3000:]


def test_forced_rccl_on_shared_gpu_fails_fast():
    """rabit_device_algo=rccl with ranks sharing one GPU: RCCL refuses that layout, so the job
    must stop at once with a clear message instead of hanging in ncclCommInitRank"""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import time
    t0 = time.time()
    rc, out = _run("device_multi.py", 2, ["rabit_device_algo=rccl"], attempts=1, timeout=120)
    assert rc != 0
    assert "no device transport" in out and "rabit_device_algo=rccl" in out, out[-3000:]
    assert time.time() - t0 < 90


def test_rccl_init_failure_falls_back_to_direct():
    """a communicator that does not come up on every rank (rabit_mock_rccl_init_fail) is an
    environment problem, not a peer failure: every rank agrees to drop RCCL and the job runs on
    the direct transport instead of looping through recovery"""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    rc, out = _run("device_multi.py", 2, ["rabit_mock_rccl_init_fail=1"], attempts=1, timeout=180)
    assert rc == 0, out[-5000:]
    assert out.count("DEVMULTI OK") == 2, out[-3000:]
    assert "running on the direct transport alone" in out, out[-3000:]


@pytest.mark.parametrize("world", [4, 8])
def test_small_op_stress(world):
    """thousands of back-to-back small allreduces (fused one-shot, classic one-shot, two-shot),
    values changing every op, results checked: a rank overwriting a stage buffer a slower peer
    still reads would show up as a wrong sum"""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    rc, out = _run("oneshot_stress.py", world, ["1500", "rabit_device_fused=1"], timeout=240)
    assert rc == 0, out[-5000:]
    assert out.count("STRESS OK") == world, out[-3000:]
