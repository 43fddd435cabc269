"""BASELINE config 5: fault-tolerant iterations — a 256 MiB Sum allreduce plus a CheckPoint every
iteration, with one worker killed mid-run by the mock engine and recovered.

    python -m rabit_amd.launcher -n 4 --num-attempt 2 python tools/robust_bench.py mock=3,4,0,0

Each iteration of every rank: grad = model * 1e-3 + rank (HBM), allreduce(grad, SUM) on the
device plane, model += grad, checkpoint_tensors({model}) (HBM snapshot + async pinned mirror).
Without a GPU the same loop runs on numpy arrays over TCP (16 MiB).  The mock key
`mock=r,v,s,t` kills rank r at its s-th collective after checkpoint v (trial t); the launcher
restarts it, it reloads the model from a survivor's snapshot and replays what it missed.

Every rank prints one JSON line: per-iteration wall times, time spent in checkpoints, and —
for the restarted rank — the time from process start to being back in step.  Rank 0's line
carries the summary (steady-state iteration median, the slowest iteration = the one that
absorbed the failure).
"""
import json
import os
import sys
import time

import numpy as np

T_START = time.time()
import rabit_amd as rabit  # noqa: E402


def process_created():
    """epoch time this process was created, to the kernel's clock tick (psutil's create_time
    rounds the boot time to whole seconds)"""
    with open("/proc/self/stat") as f:
        start_ticks = int(f.read().rsplit(")", 1)[1].split()[19])  # field 22: starttime
    with open("/proc/uptime") as f:
        up = float(f.read().split()[0])
    return time.time() - (up - start_ticks / os.sysconf("SC_CLK_TCK"))


def main():
    args = [a for a in sys.argv[1:] if "=" in a]
    iters = int(os.environ.get("XR_ITERS", "10"))
    try:
        import torch
        gpu = torch.cuda.is_available()
    except ImportError:
        gpu = False
    rabit.init(args, lib="mock", **({"rabit_device": 0} if gpu else {}))
    rank, world = rabit.get_rank(), rabit.get_world_size()
    attempt = int(os.environ.get("DMLC_NUM_ATTEMPT", "0"))
    nbytes = (256 << 20) if gpu else (16 << 20)
    n = nbytes // 4
    if gpu:
        dev = torch.device("cuda", 0)
        model = torch.zeros(n, device=dev)
        version, meta = rabit.load_checkpoint_tensors({"model": model})
    else:
        version, state = rabit.load_checkpoint()
        model = state if version else np.zeros(n, dtype=np.float32)
    t_loaded = time.time()
    iter_t, ckpt_t, iter_t0 = [], [], []
    for it in range(version, iters):
        t0 = time.time()
        iter_t0.append(t0)
        if gpu:
            grad = model * 1e-3 + rank
            rabit.allreduce(grad, rabit.SUM)
            model.add_(grad)
            torch.cuda.current_stream().synchronize()
        else:
            grad = model * 1e-3 + rank
            grad = rabit.allreduce(grad, rabit.SUM)
            model += grad
        t1 = time.time()
        if gpu:
            rabit.checkpoint_tensors({"model": model}, meta={"it": it + 1})
            torch.cuda.current_stream().synchronize()
        else:
            rabit.checkpoint(model)
        t2 = time.time()
        iter_t.append(t2 - t0)
        ckpt_t.append(t2 - t1)
    # closed form check: the model stays uniform and every iteration maps m to
    # m * (1 + 1e-3 * world) + world * (world - 1) / 2 (a wrong replay after the failure shows)
    expect = 0.0
    for _ in range(iters):
        expect = expect * (1.0 + 1e-3 * world) + world * (world - 1) / 2.0
    if gpu:
        lo, hi = float(model.min().item()), float(model.max().item())
    else:
        lo, hi = float(model.min()), float(model.max())
    model_ok = abs(lo - expect) <= 1e-4 * expect and abs(hi - expect) <= 1e-4 * expect
    st = rabit.stats()
    # recovery cost, split (stats()["recovery_phases_s"]); the restarted rank's process start-up
    # (interpreter, imports, rabit.init) is reported apart: it is the launcher's and Python's
    ph = st.get("recovery_phases_s", {})
    startup = ph.get("process_start_to_init", 0.0) if attempt > 0 else 0.0
    startup = float(rabit.allreduce(np.array([startup]), rabit.MAX)[0])
    worst = float(rabit.allreduce(np.array([max(iter_t) if iter_t else 0.0]), rabit.MAX)[0])
    # the restart timeline (epoch seconds): when the failure iteration began on the survivors,
    # when the replacement process was created, when it had loaded its checkpoint, and its own
    # first iteration
    created = process_created() if attempt > 0 else 0.0
    fail_t0 = iter_t0[int(np.argmax(iter_t))] if iter_t and attempt == 0 else 0.0
    tl = rabit.allreduce(np.array([created, t_loaded if attempt > 0 else 0.0,
                                   iter_t[0] if iter_t and attempt > 0 else 0.0, fail_t0]),
                         rabit.MAX)
    rec = {"rank": rank, "world": world, "attempt": attempt, "device": gpu,
           "bytes": nbytes, "start_version": version,
           "iter_ms": [round(t * 1e3, 2) for t in iter_t],
           "checkpoint_ms": [round(t * 1e3, 3) for t in ckpt_t],
           "recoveries": st["n_recover_events"], "recovered_ops": st["n_recovered_ops"],
           "device_replays": st.get("n_device_replays", 0),
           "model_check": {"ok": model_ok, "expect": expect, "min": lo, "max": hi},
           "recovery_phases_s": ph}
    if attempt > 0:
        rec["restart_to_loaded_s"] = round(t_loaded - T_START, 3)
    if rank == 0 and iter_t:
        steady = sorted(iter_t)[: max(1, len(iter_t) - 2)]
        rec["summary"] = {"steady_iter_ms_median": round(float(np.median(steady)) * 1e3, 2),
                          "slowest_iter_ms": round(max(iter_t) * 1e3, 2),
                          "checkpoint_ms_median": round(float(np.median(ckpt_t)) * 1e3, 3),
                          # the iteration that absorbed the failure (max over ranks), less the
                          # restarted process's start-up to rabit.init()
                          "failure_iter_ms_max_over_ranks": round(worst * 1e3, 2),
                          "restarted_startup_to_init_ms": round(startup * 1e3, 2),
                          "failure_iter_minus_startup_ms": round((worst - startup) * 1e3, 2)}
        if tl[0] > 0:
            # failure iteration = respawn + start-up to init + init to loaded + the
            # replacement's first iteration (+ the survivors' own wait to finish it)
            rec["summary"]["restart_timeline_ms"] = {
                "iteration_start_to_respawn": round((tl[0] - tl[3]) * 1e3, 1),
                "respawn_to_init": round(startup * 1e3, 1),
                "init_to_checkpoint_loaded": round((tl[1] - tl[0] - startup) * 1e3, 1),
                "restarted_first_iteration": round(tl[2] * 1e3, 1)}
    print("ROBUST " + json.dumps(rec), flush=True)
    rabit.finalize()
    if not model_ok:
        sys.exit("rank %d: model %.6g..%.6g, expected %.6g" % (rank, lo, hi, expect))


if __name__ == "__main__":
    main()
