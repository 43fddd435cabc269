#!/usr/bin/env python3
"""Headline benchmark of xrabit on MI355X (BASELINE.json): 128 MB float32 Allreduce<Sum>.

Each timed step is one `rabit.allreduce(x, SUM)` of a 128 MB float32 HBM tensor (a plain torch
allocation, as a training job's gradient) through the fault-tolerant (robust) engine: the
collective over xGMI (RCCL or the direct IPC transport, whichever the start-up calibration
measured faster) written straight into the HBM result log and the user tensor.  Nothing is
skipped.

At N > 1 the run also times every transport the job has up, side by side, on torch-allocated
and on symmetric-heap inputs (RCCL; direct pull and push, each as one fused kernel per chunk and
in the classic 5-launch form), each first checked bit for bit against a host fp64 reference.
At N = 1 no byte moves between ranks: the step is the robust
engine's bookkeeping plus its HBM result-log copy (rabit_world1_fastpath=0), reported as such
(`collective: false`); busbw is 0 by definition.

    python bench.py                       # N=1
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
        --master-port 29500 bench.py --gpus 8

Rank 0 prints one JSON line.  `value` is BASELINE.json's metric, the allreduce BUS bandwidth
(nccl-tests: busbw = algbw * 2(N-1)/N, algbw = S / t, S = 128 MiB per rank, weak scaling) at
N > 1.  At N = 1 busbw is 0 by definition (no byte crosses a link), so `value` is the algbw of
the robust engine's local op and `collective` is false; `value_is` names which one it is.  The
per-step wall clock, algbw, the whole-job aggregate N * S / t and the reference's own
`sum_tdiff-speed` (per-rank MiB/s, test/speed_test.cc:52-69) are reported alongside.  The whole
run is under a wall-clock deadline (--deadline): a rank that exceeds it names the phase it was in
and exits non-zero.  The side
measurements after the headline (variants, extras) have a budget of their own (--post-deadline)
and cannot take the measured headline with them: an exception in one is recorded in
`post_headline_failure`, and a rank stuck in one ends the run with the headline printed.
"""
import argparse
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PHASE = {"name": "start", "t0": time.time()}


def phase(name):
    PHASE["name"] = name


def start_deadline(seconds, rank, post_seconds):
    """exit non-zero, naming the phase, if the run is not done within `seconds`.  Once the
    headline is measured (HEADLINE["rec"] set), the phases after it (variants, extras) get
    `post_seconds` more at most; if they overrun, or a rank hangs in them, rank 0 still prints
    the measured headline once (flagged with the phase that did not finish) and the run exits 0:
    a broken side measurement must not take the headline with it."""
    def watch():
        while True:
            now = time.time()
            rec = HEADLINE["rec"]
            limit = PHASE["t0"] + seconds
            if rec is not None:
                limit = min(limit, HEADLINE["t"] + post_seconds)
            if now >= limit:
                break
            time.sleep(min(1.0, limit - now))
        sys.stderr.write("bench.py: rank %d exceeded its deadline in phase '%s' "
                         "(%.0f s into the run)\n"
                         % (rank, PHASE["name"], time.time() - PHASE["t0"]))
        sys.stderr.flush()
        if HEADLINE["rec"] is not None:
            emit_headline("deadline in phase '%s'" % PHASE["name"])
            os._exit(0)
        os._exit(3)
    t = threading.Thread(target=watch, daemon=True)
    t.start()
    return t


HEADLINE = {"rec": None, "t": 0.0, "printed": False, "rank": 0}
PRINT_LOCK = threading.Lock()


def emit_headline(failure=None):
    """rank 0 prints the one JSON line, exactly once (main thread or deadline watcher)"""
    with PRINT_LOCK:
        if HEADLINE["printed"] or HEADLINE["rec"] is None:
            return
        HEADLINE["printed"] = True
        rec = HEADLINE["rec"]
        if failure is not None:
            rec["post_headline_failure"] = failure
        if HEADLINE["rank"] == 0:
            print(json.dumps(rec), flush=True)


def pattern_fill(x, rank):
    """exactly representable float32 data: x[i] = (7 i + 13 rank) mod 1024, so every order of
    summation over <= 8 ranks gives the same bits"""
    import torch
    i = torch.arange(x.numel(), device=x.device, dtype=torch.int64)
    x.copy_(((i * 7 + 13 * rank) % 1024).to(x.dtype))


def host_reference(n, world):
    """fp64 sum over ranks of pattern_fill, on the host"""
    i = np.arange(n, dtype=np.int64)
    acc = np.zeros(n, dtype=np.float64)
    for r in range(world):
        acc += ((i * 7 + 13 * r) % 1024).astype(np.float64)
    return acc


def check_allreduce(rabit, x, rank, ref):
    """one allreduce of the pattern, compared element by element with the host reference;
    the verdict is agreed over all ranks (max of the failure flags)"""
    pattern_fill(x, rank)
    rabit.allreduce(x, rabit.SUM)
    ok = bool(np.array_equal(x.cpu().numpy().astype(np.float64), ref))
    bad = rabit.allreduce(np.array([0 if ok else 1], dtype=np.int32), rabit.MAX)[0]
    return not bad


def _timed(rabit, torch, fn, reps, settle=0.0, device_wide=True):
    """median wall time (s) of fn() over reps, ranks in lock step, max over ranks.
    device_wide=False waits for the caller's stream only (work the library leaves running on
    its own side streams, like a checkpoint's host mirror, is not on the caller's path)"""
    times = []
    for _ in range(reps):
        if settle:
            time.sleep(settle)  # e.g. let the previous checkpoint's host mirror finish
        torch.cuda.synchronize()
        rabit.allreduce(np.zeros(1, dtype=np.int32), rabit.SUM)
        t0 = time.perf_counter()
        fn()
        if device_wide:
            torch.cuda.synchronize()
        else:
            torch.cuda.current_stream().synchronize()
        times.append(time.perf_counter() - t0)
    med = float(np.median(times))
    return float(rabit.allreduce(np.array([med]), rabit.MAX)[0])


def reference_measured(world, value):
    """The reference's own speed_test built from its sources and run on the host of an MI355X
    box (tools/refbuild/, profiles/r1_h2h_reference/): its Sum time for the same 128 MiB float32
    job at this world size, as the same whole-job aggregate.  BASELINE.md publishes no number,
    so `vs_baseline` stays null; this is a measured comparison with its provenance."""
    path = os.path.join(ROOT, "profiles", "r1_h2h_reference", "h2h_128MiB.jsonl")
    try:
        rows = [json.loads(l) for l in open(path) if l.strip()]
    except OSError:
        return None
    for r in rows:
        if r.get("impl") == "reference" and r.get("world") == world and r.get("rc") == 0:
            if world == 1:
                return {"note": "the reference's robust engine returns without work at world 1",
                        "source": os.path.relpath(path, ROOT)}
            t = r["sum_mean_s"] / r["nrep"]
            ref_value = world * r["bytes"] / t / 1e9
            return {"value": round(ref_value, 3), "unit": "GB/s", "ms_per_op": round(t * 1e3, 2),
                    "data_path": "host memory over TCP (its only path)",
                    "vs_reference_measured": round(value / ref_value, 1),
                    "source": os.path.relpath(path, ROOT)}
    return None


def calibrated_mode(st):
    """the direct form the calibration chose, as set_device_transport names it"""
    if st.get("direct_pipeline"):
        return "pipelined"
    return "push" if st.get("direct_push") else "pull"


def size_sweep(rabit, torch, dev, world):
    """N > 1: float32 sum latency from 4 KiB to 128 MiB on each transport and direct form that
    is up (median of 10, ranks in lock step, max over ranks), and on the calibrated routing --
    the data behind the size routing.  routed_over_best: the routed time over the best forced
    variant per size (1.0 = the routing picked the fastest).  The calibrated routing is restored
    afterwards."""
    out = {}
    sizes = (4 << 10, 64 << 10, 1 << 20, 4 << 20, 16 << 20, 32 << 20, 128 << 20)
    legs = (("rccl", rabit.TRANSPORT_RCCL, None), ("direct-pull", rabit.TRANSPORT_DIRECT, "pull"),
            ("direct-push", rabit.TRANSPORT_DIRECT, "push"),
            ("direct-pipelined", rabit.TRANSPORT_DIRECT, "pipelined"),
            ("routed", rabit.TRANSPORT_AUTO, None))
    xs = {nb: torch.ones(nb // 4, dtype=torch.float32, device=dev) for nb in sizes}
    for name, which, mode in legs:
        phase("sweep %s" % name)
        up = rabit.set_device_transport(which, mode)
        up = not rabit.allreduce(np.array([0 if up else 1], dtype=np.int32), rabit.MAX)[0]
        if not up:
            continue
        row = {}
        for nbytes in sizes:
            x = xs[nbytes]
            rabit.allreduce(x, rabit.SUM)
            row[str(nbytes)] = round(_timed(rabit, torch, lambda: rabit.allreduce(x, rabit.SUM),
                                            10) * 1e6, 1)
            rabit.checkpoint(None)
        out[name + "_us"] = row
    rabit.set_device_transport(rabit.TRANSPORT_AUTO, None)
    del xs
    routed = out.get("routed_us")
    if routed:
        ratio = {}
        for k, t in routed.items():
            best = min([v[k] for n, v in out.items() if n != "routed_us" and k in v] or [t])
            ratio[k] = round(t / best, 3) if best > 0 else None
        out["routed_over_best"] = ratio
    return out


def run_extras(rabit, torch, dev, world):
    """BASELINE.json configs 3 and 4 plus the checkpoint cost of config 5, on this job's ranks
    (result log and checkpoint paths included, as in the headline step)."""
    out = {}
    if world > 1:
        # xGMI per-link and all-link bandwidth, reads / writes / both ways (direct transport's
        # IPC mappings; on ranks sharing one GPU this is HBM): min over ranks
        phase("link probe")
        try:
            lp = rabit.link_probe(64 << 20)
        except RuntimeError as e:  # a failed probe costs its own numbers, not the other extras
            lp = None
            out["link_probe_error"] = str(e)
        ok = rabit.allreduce(np.array([0 if lp is None else 1], dtype=np.int32), rabit.MIN)[0]
        if ok:
            keys = sorted(lp)
            low = rabit.allreduce(np.array([lp[k] for k in keys]), rabit.MIN)
            out["link_probe_min_over_ranks"] = {k: round(float(v), 2) for k, v in zip(keys, low)}
        out["size_sweep"] = size_sweep(rabit, torch, dev, world)
    # the reference speed_test's whole line: Max, Sum and a random-root Broadcast per repetition
    phase("speed_test line")
    out["speed_test"] = speed_test_line(rabit, torch, dev, world, (128 << 20) // 4)
    # config 3: Broadcast of a 1 GiB blob from root 0
    nb = 1 << 30
    blob = torch.empty(nb, dtype=torch.uint8, device=dev)
    if rabit.get_rank() == 0:
        blob.fill_(7)
    rabit.broadcast_tensor(blob, 0)
    ok = bool((blob[:: 1 << 20] == 7).all().item())
    t = _timed(rabit, torch, lambda: rabit.broadcast_tensor(blob, 0), 3)
    out["broadcast_1GiB_ms"] = round(t * 1e3, 3)
    out["broadcast_1GiB_busbw_GBps"] = round(nb / t / 1e9, 2) if world > 1 else None
    out["broadcast_check"] = ok
    if world > 1:
        # the same broadcast on each transport that is up (the routed one above is the
        # broadcast calibration's choice), each checked
        st0 = rabit.stats()
        per = {}
        for name, which in (("rccl", rabit.TRANSPORT_RCCL), ("direct", rabit.TRANSPORT_DIRECT)):
            phase("broadcast %s" % name)
            up = rabit.set_device_transport(which, None)
            up = not rabit.allreduce(np.array([0 if up else 1], dtype=np.int32), rabit.MAX)[0]
            if not up:
                continue
            blob.fill_(7 if rabit.get_rank() == 0 else 0)
            rabit.broadcast_tensor(blob, 0)
            good = bool((blob[:: 1 << 20] == 7).all().item())
            tt = _timed(rabit, torch, lambda: rabit.broadcast_tensor(blob, 0), 3)
            per[name] = {"ms": round(tt * 1e3, 3), "busbw_GBps": round(nb / tt / 1e9, 2),
                         "check": good}
            rabit.checkpoint(None)
        rabit.set_device_transport(rabit.TRANSPORT_AUTO, None)
        out["broadcast_1GiB_by_transport"] = per
        st1 = rabit.stats()
        out["broadcast_routing"] = {"calibration_us": dict(zip(
            ["rccl_64KiB", "rccl_big", "direct_64KiB", "direct_big"],
            st1.get("calib_bcast_us", []))),
            "direct_min_bytes": st1.get("bcast_direct_min"),
            "direct_below_bytes": st1.get("bcast_direct_below"),
            "direct_bcast_chunks": st1.get("direct_bcast_chunks")}
    del blob
    rabit.checkpoint(None)  # clears the result log (keeps HBM use bounded)
    # config 4: lazy allreduce, prepare = per-element squared gradient, 64 MiB
    n = (64 << 20) // 4
    grad = torch.rand(n, dtype=torch.float32, device=dev)
    acc = torch.empty_like(grad)

    def fused():
        rabit.allreduce_prepared(acc, grad, rabit.SUM, rabit.PREP_SQUARE)

    def unfused():
        torch.mul(grad, grad, out=acc)
        rabit.allreduce(acc, rabit.SUM)

    fused()
    unfused()
    out["lazy_sq_64MiB_fused_us"] = round(_timed(rabit, torch, fused, 5) * 1e6, 1)
    out["lazy_sq_64MiB_unfused_us"] = round(_timed(rabit, torch, unfused, 5) * 1e6, 1)
    rabit.checkpoint(None)
    del grad, acc
    # the headline's 128 MiB as bf16 gradients (extended dtype; fp32 accumulation in the kernels)
    hb = torch.rand((128 << 20) // 2, device=dev).to(torch.bfloat16)
    rabit.allreduce(hb, rabit.SUM)
    t = _timed(rabit, torch, lambda: rabit.allreduce(hb, rabit.SUM), 5)
    out["allreduce_128MiB_bf16_us"] = round(t * 1e6, 1)
    out["allreduce_128MiB_bf16_busbw_GBps"] = (
        round((128 << 20) / t / 1e9 * 2 * (world - 1) / world, 2) if world > 1 else None)
    rabit.checkpoint(None)
    del hb
    # the reference's own benchmark shape (test/speed_test.cc): 128 MiB float32 in HOST memory.
    # Under torchrun large host allreduces go through HBM (rabit_host_via_device), pipelined
    # through pinned slots (host_stager.h); at N = 1 it is the robust engine's host path.
    phase("host buffer")
    hn = (128 << 20) // 4
    hx = torch.empty(hn, dtype=torch.float32)  # host memory, reduced in place (no copy)
    hx.copy_(torch.from_numpy(((np.arange(hn, dtype=np.int64) * 7 + 13 * rabit.get_rank())
                               % 1024).astype(np.float32)))
    rabit.allreduce(hx, rabit.SUM)
    host_ok = bool(np.array_equal(hx.numpy().astype(np.float64), host_reference(hn, world)))
    th = []
    for _ in range(3):
        hx.fill_(1.0)
        rabit.allreduce(np.zeros(1, dtype=np.int32), rabit.SUM)
        t0 = time.perf_counter()
        rabit.allreduce(hx, rabit.SUM)
        th.append(time.perf_counter() - t0)
    t = float(rabit.allreduce(np.array([float(np.median(th))]), rabit.MAX)[0])
    st_h = rabit.stats()
    out["host_buffer_128MiB_ms"] = round(t * 1e3, 2)
    out["host_buffer_128MiB_speed_MiBps"] = round((128 << 20) / t / 2 ** 20, 1)
    out["host_buffer_check"] = host_ok
    # N > 1: through HBM, whole copies or pipelined as the job's timed choice found (the first
    # ops of the job are that choice's warm-up and samples)
    out["host_buffer_path"] = ("hbm, %s" % st_h.get("host_stage_choice") if world > 1 else "host")
    out["host_buffer_stage_threads"] = st_h.get("host_stage_threads")
    rabit.checkpoint(None)
    del hx
    # config 5: 256 MiB sum + checkpoint every iteration, against the sum alone
    out.update(run_config5(rabit, torch, dev))
    rabit.checkpoint(None)
    # config 5 (checkpoint part alone): HBM snapshot of a 256 MiB model
    model = torch.rand((256 << 20) // 4, dtype=torch.float32, device=dev)
    rabit.checkpoint_tensors({"w": model}, meta={"it": 0})
    # iterations longer than the async D2H mirror (~5 ms for 256 MiB) see only the snapshot
    t = _timed(rabit, torch, lambda: rabit.checkpoint_tensors({"w": model}, meta={"it": 1}), 5,
               settle=0.05, device_wide=False)
    out["checkpoint_256MiB_us"] = round(t * 1e6, 1)
    del model
    return out


def bandwidths(world, size_bytes, t_step):
    """the headline numbers of one timed step of t_step seconds: nccl-tests algbw / busbw, the
    whole-job aggregate, and `value` (busbw at N > 1; algbw at N = 1, where busbw is 0)"""
    algbw = size_bytes / t_step / 1e9
    busbw = algbw * (2.0 * (world - 1) / world) if world > 1 else 0.0
    out = {"algbw_GBps": round(algbw, 2), "busbw_GBps": round(busbw, 2),
           "aggregate_GBps": round(world * size_bytes / t_step / 1e9, 2)}
    if world > 1:
        out["value"], out["value_is"] = out["busbw_GBps"], "busbw_GBps"
    else:
        out["value"] = out["algbw_GBps"]
        out["value_is"] = "algbw_GBps (N=1: busbw is 0 by definition)"
    return out


def time_steps(rabit, torch, x, steps, with_mean=False):
    """wall time of `steps` back-to-back allreduces, ranks in lock step, max over ranks
    (with_mean: also the mean over ranks, as the reference's speed_test averages)"""
    torch.cuda.synchronize()
    rabit.allreduce(np.zeros(1, dtype=np.int32), rabit.SUM)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        rabit.allreduce(x, rabit.SUM)
    torch.cuda.synchronize()
    rabit.allreduce(np.zeros(1, dtype=np.int32), rabit.SUM)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    worst = float(rabit.allreduce(np.array([elapsed]), rabit.MAX)[0])
    if not with_mean:
        return worst
    mean = float(rabit.allreduce(np.array([elapsed]), rabit.SUM)[0]) / rabit.get_world_size()
    return worst, mean


def measure_ft_tax(rabit, torch, x, steps, t_robust):
    """What fault tolerance costs on the headline op: the same 128 MiB sum on the same
    transport and routing through rabit.probe_allreduce (outside the result log and the
    sequence numbering), in place with the host wait as the base engine runs it, with the
    robust engine's dual store (log slot + user buffer), and stream-ordered without the host
    wait.  ft_tax = robust step - base op; the other two split it.  Ranks in lock step, max over
    ranks (as time_steps)."""
    out = {}
    for name, mode in (("base_us", rabit.PROBE_BASE), ("dual_store_us", rabit.PROBE_DUAL_STORE),
                       ("no_host_wait_us", rabit.PROBE_NO_WAIT)):
        phase("ft tax %s" % name)
        for _ in range(2):
            rabit.probe_allreduce(x, rabit.SUM, mode)
        torch.cuda.synchronize()
        rabit.allreduce(np.zeros(1, dtype=np.int32), rabit.SUM)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            rabit.probe_allreduce(x, rabit.SUM, mode)
        torch.cuda.synchronize()
        rabit.allreduce(np.zeros(1, dtype=np.int32), rabit.SUM)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        out[name] = round(float(rabit.allreduce(np.array([el]), rabit.MAX)[0]) / steps * 1e6, 1)
    t_base = out["base_us"]
    out["robust_us"] = round(t_robust * 1e6, 1)
    out["ft_tax_us"] = round(t_robust * 1e6 - t_base, 1)
    out["ft_tax_pct"] = round(100.0 * (t_robust * 1e6 - t_base) / (t_robust * 1e6), 1)
    out["dual_store_cost_us"] = round(out["dual_store_us"] - t_base, 1)
    out["host_wait_cost_us"] = round(t_base - out["no_host_wait_us"], 1)
    out["definition"] = ("robust = the headline step; base = the same op in place with the host "
                         "wait, outside the result log; dual_store = into a log-like slot and the "
                         "user buffer; no_host_wait = in place, stream-ordered")
    return out


def speed_test_line(rabit, torch, dev, world, n, nrep=5):
    """The reference speed_test's whole output line (test/speed_test.cc:13-99) on HBM buffers:
    per repetition Allreduce<Max> of n float32, Allreduce<Sum> of n float32 and a Broadcast of
    n bytes from a random root (srand(0); rand() % nproc), each rank summing its own time per
    kind; then mean / std over ranks and speed = n * nrep * sizeof(T) / mean / 2^20 (MiB/s per
    rank), as its PrintStats."""
    rng = np.random.RandomState(0)
    rank = rabit.get_rank()
    i = torch.arange(n, device=dev, dtype=torch.int64)
    mx = ((i * (rank + 1)) % 111).to(torch.float32)
    sm = ((i * (rank + 1)) % 131).to(torch.float32)
    bc = torch.empty(n, dtype=torch.uint8, device=dev)
    del i
    td = {"max_tdiff": 0.0, "sum_tdiff": 0.0, "bcast_tdiff": 0.0}

    def timed(key, fn):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        td[key] += time.perf_counter() - t0
    # one untimed round (transport bring-up, first touches), as the headline's warm-up
    rabit.allreduce(mx, rabit.MAX)
    rabit.allreduce(sm, rabit.SUM)
    rabit.broadcast_tensor(bc, 0)
    rabit.checkpoint(None)
    t_start = time.perf_counter()
    for _ in range(nrep):
        root = int(rng.randint(0, 2 ** 31 - 1)) % world
        timed("max_tdiff", lambda: rabit.allreduce(mx, rabit.MAX))
        timed("sum_tdiff", lambda: rabit.allreduce(sm, rabit.SUM))
        timed("bcast_tdiff", lambda: rabit.broadcast_tensor(bc, root))
    td["tot_tdiff"] = time.perf_counter() - t_start
    out = {}
    for key, size in (("max_tdiff", 4), ("sum_tdiff", 4), ("bcast_tdiff", 1), ("tot_tdiff", 0)):
        tavg = float(rabit.allreduce(np.array([td[key]]), rabit.SUM)[0]) / world
        tsqr = float(rabit.allreduce(np.array([(td[key] - tavg) ** 2]), rabit.SUM)[0])
        rec = {"mean_s": round(tavg, 6), "std_s": round(float(np.sqrt(tsqr / world)), 6)}
        if size:
            rec["speed_MiBps"] = round(n * nrep * size / tavg / 2 ** 20, 1)
        out[key] = rec
    out["n"], out["nrep"], out["buffers"] = n, nrep, "HBM (torch)"
    rabit.checkpoint(None)
    return out


def run_config5(rabit, torch, dev, iters=5):
    """BASELINE.json config 5 without the kill: every iteration allreduces a 256 MiB float32
    gradient through the robust engine, applies it to a 256 MiB model and checkpoints the model
    (HBM snapshot + async host mirror, reference flow src/allreduce_robust.cc:484-557).  The
    same loop without the checkpoint gives the checkpoint's overhead.  Ranks in lock step, median
    iteration, max over ranks.  The kill/recover timing is tools/robust_bench.py's job."""
    n = (256 << 20) // 4
    grad = torch.rand(n, dtype=torch.float32, device=dev).mul_(1e-3)
    model = torch.zeros(n, dtype=torch.float32, device=dev)
    it = [0]

    def step(ckpt):
        rabit.allreduce(grad, rabit.SUM)
        model.add_(grad, alpha=-1e-3)
        if ckpt:
            it[0] += 1
            rabit.checkpoint_tensors({"w": model}, meta={"it": it[0]})

    step(True)
    # the iteration ends when the caller's stream is done: the checkpoint's host mirror runs on
    # the library's side stream (SDMA / copy engine) behind the next iteration, as in training
    t_ckpt = _timed(rabit, torch, lambda: step(True), iters, device_wide=False)
    # the same, waiting for every stream of the device (the host mirror of 256 MiB included)
    t_drained = _timed(rabit, torch, lambda: step(True), iters)
    # the same iterations without the checkpoint (their results stay in the HBM log until the
    # checkpoint after the loop: iters x 256 MiB)
    step(False)
    t_sum = _timed(rabit, torch, lambda: step(False), iters, device_wide=False)
    rabit.checkpoint(None)
    del grad, model
    return {"config5_iter_us": round(t_ckpt * 1e6, 1),
            "config5_sum_only_iter_us": round(t_sum * 1e6, 1),
            "config5_ckpt_overhead_us": round((t_ckpt - t_sum) * 1e6, 1),
            "config5_iter_mirror_drained_us": round(t_drained * 1e6, 1), "config5_iters": iters}


def run_variants(rabit, torch, dev, n, world, rank, ref, steps, forced_rccl=False):
    """every transport this job has up, on torch-allocated and symmetric-heap inputs: time
    and busbw of the 128 MiB float32 sum, each checked against the host fp64 reference; plus
    the per-phase times of the classic direct form (pull and push)"""
    out = []
    bufs = [("torch", torch.empty(n, dtype=torch.float32, device=dev))]
    try:
        bufs.append(("symmetric", rabit.symmetric_empty(n, torch.float32)))
    except MemoryError:
        pass
    variants = [("rccl", rabit.TRANSPORT_RCCL, None, None)]
    for mode in ("pull", "push"):
        for fused in (False, True):
            variants.append(("direct-%s-%s" % (mode, "fused" if fused else "classic"),
                             rabit.TRANSPORT_DIRECT, mode, fused))
    # the push of chunk k and the gather of chunk k-2 in one round (opposite link directions)
    variants.append(("direct-push-pipelined", rabit.TRANSPORT_DIRECT, "pipelined", False))
    st0 = rabit.stats()
    for input_name, x in bufs:
        for name, which, mode, fused in variants:
            phase("variant %s/%s" % (name, input_name))
            up = rabit.set_device_transport(which, mode, fused)
            # the same choice on every rank, or none
            up = not rabit.allreduce(np.array([0 if up else 1], dtype=np.int32), rabit.MAX)[0]
            rec = {"transport": name, "input": input_name, "available": bool(up)}
            if up:
                rec["check"] = check_allreduce(rabit, x, rank, ref)
                x.copy_(torch.rand(n, device=dev).mul_(1e-3))
                for _ in range(2):
                    rabit.allreduce(x, rabit.SUM)
                t = time_steps(rabit, torch, x, steps) / steps
                rec["t_us"] = round(t * 1e6, 1)
                rec["algbw_GBps"] = round(n * 4 / t / 1e9, 2)
                rec["busbw_GBps"] = round(n * 4 / t / 1e9 * 2 * (world - 1) / world, 2)
                rabit.checkpoint(None)  # bounded result log
            out.append(rec)
    # where the time of the classic direct form goes (stage copy, barriers, reduce, gather),
    # per phase from hipEvents, on the torch-allocated input: evidence for tuning the xGMI path
    x = bufs[0][1]
    phases = []
    for mode in ("pull", "push"):
        phase("phases %s" % mode)
        up = rabit.set_device_transport(rabit.TRANSPORT_DIRECT, mode, False)
        up = not rabit.allreduce(np.array([0 if up else 1], dtype=np.int32), rabit.MAX)[0]
        if not up:
            continue
        rabit.set_phase_timing(True)
        for _ in range(5):
            rabit.allreduce(x, rabit.SUM)
        torch.cuda.synchronize()
        st = rabit.stats()
        rabit.set_phase_timing(False)
        phases.append({"transport": "direct-%s-classic" % mode, "input": "torch",
                       "phase_us": st.get("direct_phase_us"),
                       "timed_ops": st.get("direct_timed_ops")})
        rabit.checkpoint(None)
    # back to the calibrated choice of transport and direct form (or to RCCL after a fallback)
    if forced_rccl:
        rabit.set_device_transport(rabit.TRANSPORT_RCCL, None)
        return out, phases
    rabit.set_device_transport(rabit.TRANSPORT_AUTO, None)
    return out, phases


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--size-mb", type=int, default=128)
    ap.add_argument("--engine", default="robust", choices=["robust", "base"])
    ap.add_argument("--check", type=int, default=1, help="verify one reduction first")
    ap.add_argument("--symmetric", type=int, default=0,
                    help="1: the headline buffer lives in rabit's symmetric heap (IPC-registered "
                         "HBM the direct transport reads in place, like registered buffers in "
                         "nccl-tests); 0 (default): a plain torch allocation")
    ap.add_argument("--variants", type=int, default=1,
                    help="N > 1: also time every transport on torch and symmetric-heap inputs")
    ap.add_argument("--extras", type=int, default=1,
                    help="after the timed loop, also time the other BASELINE configs: 1 GiB "
                         "broadcast, 64 MiB lazy (squared-gradient) allreduce fused vs unfused, "
                         "256 MiB HBM checkpoint")
    ap.add_argument("--rccl-tune", type=int, default=1,
                    help="N > 1: time RCCL's own channel count against fixed CTA counts at "
                         "start-up and keep the fastest")
    ap.add_argument("--deadline", type=int, default=600,
                    help="wall-clock limit of the whole run in seconds")
    ap.add_argument("--post-deadline", type=int, default=240,
                    help="seconds the phases after the headline (variants, extras) may take "
                         "before rank 0 prints the headline alone and the run ends")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("bench.py --gpus %d but WORLD_SIZE=%d: launch N>1 with "
                         "torch.distributed.run" % (args.gpus, world))
    start_deadline(args.deadline, rank, args.post_deadline)
    phase("import")
    import torch
    import rabit_amd as rabit
    from rabit_amd.torchrun import init_from_env

    # one process per GPU; with fewer GPUs than ranks (a rehearsal of the N>1 launch on a
    # one-GPU box) ranks share GPUs and the direct IPC transport carries the data (RCCL refuses
    # two ranks on one GPU), which is flagged in the output
    ngpu = torch.cuda.device_count()
    gpu = local_rank % ngpu
    shared_gpu = ngpu < int(os.environ.get("LOCAL_WORLD_SIZE", world))
    torch.cuda.set_device(gpu)
    n = args.size_mb * (1 << 20) // 4
    # the symmetric heap holds the variant matrix's second buffer (+ 48 MiB of slack); the
    # calibration runs first and reads its inputs (up to 128 MiB) from the heap's free tail
    heap_bytes = n * 4 + (48 << 20) if (world > 1 and args.variants) or args.symmetric else 0
    heap = {"rabit_device_symmetric_heap": str(heap_bytes)} if heap_bytes else {}
    phase("init")
    # N > 1: RCCL's channel (CTA) count is timed at start-up against fixed counts and the
    # fastest communicator is kept (transport.rccl_tuning)
    tune = {"rabit_rccl_tune": "1"} if world > 1 and args.rccl_tune else {}
    # the robust engine logs every result until the next checkpoint: reserve the HBM log for
    # the check, warmup and timed steps up front (one allocation), as a job would size it for
    # the results of one iteration, so the timed loop never waits on hipMalloc
    # Long runs (large --steps) log more than the default 64 GiB HBM cap: let the log use this
    # rank's share of the free HBM (less 16 GiB for the heap, stages and the extras' buffers)
    # before it spills to pinned host memory, and never reserve more than that share.
    free_hbm = torch.cuda.mem_get_info(gpu)[0]
    ranks_here = max(1, -(-int(os.environ.get("LOCAL_WORLD_SIZE", world)) // ngpu))
    share = max(1 << 30, free_hbm // ranks_here - (16 << 30))
    want = (args.warmup + args.steps + 3) * n * 4
    log = {"rabit_device_log_reserve": str(min(want, share))}
    if want > (64 << 30):
        log["rabit_device_log_cap"] = str(max(64 << 30, share))
    ctx = init_from_env(lib="standard" if args.engine == "robust" else "base",
                        rabit_world1_fastpath=0, rabit_device=gpu, **heap, **tune, **log)
    dev = torch.device("cuda", gpu)

    phase("reference")
    ref = host_reference(n, world) if args.check or args.variants else None
    if args.symmetric:
        x = rabit.symmetric_empty(n, torch.float32)
    else:
        x = torch.empty(n, dtype=torch.float32, device=dev)
    checked = None
    check_fallback = None
    if args.check:
        phase("check")
        checked = check_allreduce(rabit, x, rank, ref)
        if not checked and world > 1:
            # the calibrated transport returned a wrong result: say so, and time RCCL instead
            # when it is up and correct (the same decision on every rank)
            st0 = rabit.stats()
            up = rabit.set_device_transport(rabit.TRANSPORT_RCCL, None)
            up = not rabit.allreduce(np.array([0 if up else 1], dtype=np.int32), rabit.MAX)[0]
            check_fallback = {"failed": "direct" if st0.get("device_direct") else "rccl",
                              "direct_fused": bool(st0.get("direct_fused", 0)),
                              "direct_push": bool(st0.get("direct_push", 0)),
                              "now": "rccl" if up else None}
            if up:
                checked = check_allreduce(rabit, x, rank, ref)
        if not checked:
            raise SystemExit("allreduce result check against the host fp64 reference failed")
    g = torch.Generator(device=dev)
    g.manual_seed(1234 + rank)
    # |x| ~ 1e-3 keeps repeated in-place sums finite for hundreds of 8-rank steps
    x.copy_(torch.rand((n,), generator=g, dtype=torch.float32, device=dev).mul_(1e-3))

    phase("warmup")
    for _ in range(args.warmup):
        rabit.allreduce(x, rabit.SUM)
    # the steady-state path checked as well: by now the input is read in place by the peers
    # (zero-copy registry) where the first check staged it; a wrong result turns zero copy off
    zero_copy_check = None
    if args.check and world > 1:
        phase("check after warmup")
        zero_copy_check = check_allreduce(rabit, x, rank, ref)
        if not zero_copy_check:
            rabit.set_zero_copy(0)
            if not check_allreduce(rabit, x, rank, ref):
                raise SystemExit("allreduce result check after the warm-up failed")
        x.copy_(torch.rand((n,), generator=g, dtype=torch.float32, device=dev).mul_(1e-3))
        for _ in range(2):
            rabit.allreduce(x, rabit.SUM)
    # a checkpoint (outside the timed region) empties the result log, as a training loop's
    # per-iteration checkpoint does: the timed steps' results are all the log holds
    if args.engine == "robust":
        rabit.checkpoint(None)
    phase("timed")
    elapsed, elapsed_mean = time_steps(rabit, torch, x, args.steps, with_mean=True)
    st_head = rabit.stats()

    t_step = elapsed / args.steps
    size_bytes = n * 4
    bw = bandwidths(world, size_bytes, t_step)
    st = st_head
    rec = {
        "metric": "allreduce_128MB_fp32_sum_busbw",
        "value": bw["value"],
        "unit": "GB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(t_step * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp32",
        "data": "synthetic",
        "config": {"model": "rabit Allreduce<op::Sum> float32 x 32Mi (speed_test.cc shape)",
                   "global_batch": world, "seq_len": n, "parallelism": "dp%d" % world,
                   "engine": args.engine, "size_bytes_per_rank": size_bytes,
                   "input_buffer": "symmetric heap" if args.symmetric else "torch allocation"},
        "value_is": bw["value_is"],
        "busbw_GBps": bw["busbw_GBps"],
        "algbw_GBps": bw["algbw_GBps"],
        "t_us": round(t_step * 1e6, 1),
        "aggregate_GBps": bw["aggregate_GBps"],
        # the reference's own number (test/speed_test.cc:52-69): S / mean-over-ranks time, MiB/s
        "sum_tdiff_speed_MiBps": round(size_bytes * args.steps / elapsed_mean / 2 ** 20, 1),
        "collective": world > 1,
        "value_definition": "busbw = algbw * 2(N-1)/N as nccl-tests, algbw = bytes_per_rank / "
                            "t_step (N=1: algbw); aggregate_GBps = N * bytes_per_rank / t_step",
        "baseline_note": "reference publishes no numbers (BASELINE.md)",
        "result_check": "bit-exact vs host fp64 reference" if checked else None,
        "check_fallback": check_fallback,
        "steady_state_check": (None if zero_copy_check is None else
                               ("bit-exact" if zero_copy_check
                                else "failed: zero copy turned off, then bit-exact")),
        "consensus_elided": st.get("n_consensus_elided", 0),
        "device_epoch": st.get("device_epoch", 0),
        "transport": {"rccl": st.get("device_rccl", 0), "direct": st.get("device_direct", 0),
                      "zero_copy_chunks": st.get("zero_copy_chunks", 0),
                      "zero_copy_registry": st.get("zero_copy_registry"),
                      "direct_min_bytes": st.get("device_direct_min", -1),
                      "direct_below_bytes": st.get("device_direct_below", 0),
                      "calibration_us": st.get("calib_us"),
                      "direct_variant": calibrated_mode(st),
                      "calibration_push_us": st.get("calib_push_us"),
                      "calibration_forms_us": dict(zip(
                          ["pull-classic", "pull-fused", "push-classic", "push-fused",
                           "push-pipelined"],
                          st.get("calib_forms_us", []))),
                      # every calibrated size x transport / direct form, and the routing bands
                      # built from them (engine/routing.h); {} when the job did not calibrate
                      "calibration_matrix": st.get("calib_matrix"),
                      "direct_pipeline": bool(st.get("direct_pipeline", 0)),
                      "pipelined_ops": st.get("pipelined_ops", 0),
                      "direct_fused": bool(st.get("direct_fused", 0)),
                      "fused_chunks": st.get("fused_chunks", 0),
                      "calibration_heap_inputs": bool(st.get("calib_heap_src", 0)),
                      "peer_links": st.get("peer_links"),
                      # HBM free at start-up (every process on this GPU counted) and the result
                      # log reserved from it: a log that outgrows its reserve allocates or
                      # spills inside the timed loop
                      "free_hbm_at_start_GiB": round(free_hbm / 2 ** 30, 1),
                      "log_reserve_GiB": round(int(log["rabit_device_log_reserve"]) / 2 ** 30, 2),
                      "log_spilled_results": st.get("n_spilled_results", 0),
                      "rccl_tuning": st.get("rccl_tuning")},
        "variants": None,
        "direct_phase_breakdown": None,
        "extras": None,
        "reference_measured": reference_measured(world, bw["aggregate_GBps"]),
    }
    if world == 1:
        rec["n1_note"] = ("N=1: no data moves between ranks; the step is the robust engine's "
                          "per-op bookkeeping plus its HBM result-log copy (robust-path overhead, "
                          "not a collective)")
    if shared_gpu:
        rec["shared_gpu_rehearsal"] = ("%d ranks on %d GPU(s): not an xGMI measurement"
                                       % (world, ngpu))
    HEADLINE["rank"] = rank
    HEADLINE["t"] = time.time()
    HEADLINE["rec"] = rec
    ft_tax = None
    if args.engine == "robust" and args.extras:
        # the fault-tolerance tax of the headline op, on the routing the headline used
        try:
            rabit.set_error_mode(True)
            rabit.checkpoint(None)
            ft_tax = measure_ft_tax(rabit, torch, x, max(5, args.steps // 2), t_step)
        except Exception as e:  # noqa: BLE001 - reported in the record
            ft_tax = {"error": "%s: %s" % (type(e).__name__, e)}

    # side measurements after the headline: an exception is recorded, not fatal (a rank stuck
    # in one is cut off by the post-headline deadline, which still prints the headline)
    # native errors raise from here on instead of exiting the process (set_error_mode)
    failures = []
    rabit.set_error_mode(True)
    if world > 1 and args.variants:
        phase("variants")
        try:
            rabit.checkpoint(None)
            rec["variants"], rec["direct_phase_breakdown"] = run_variants(
                rabit, torch, dev, n, world, rank, ref, max(5, args.steps // 2),
                forced_rccl=check_fallback is not None)
        except Exception as e:  # noqa: BLE001 - reported in the record
            failures.append("variants: %s: %s" % (type(e).__name__, e))
    if args.extras and failures:
        failures.append("extras: skipped after the variants failed")
    elif args.extras:
        phase("extras")
        try:
            rec["extras"] = run_extras(rabit, torch, dev, world)
            if ft_tax is not None:
                rec["extras"]["ft_tax"] = ft_tax
            lp = rec["extras"].get("link_probe_min_over_ranks")
            if lp and lp.get("all_links_read_GBps"):
                # the pull two-shot brings 2(n-1)/n of the buffer into every rank, so its busbw is
                # bounded by the rate at which one rank reads from all its peers at once; the push
                # forms send half of it out instead, so with them the ratio can pass 1
                rec["extras"]["busbw_over_all_links_read"] = round(
                    rec["busbw_GBps"] / lp["all_links_read_GBps"], 3)
        except Exception as e:  # noqa: BLE001
            failures.append("extras: %s: %s" % (type(e).__name__, e))
    emit_headline("; ".join(failures) if failures else None)
    phase("finalize")
    del x
    ctx.finalize()


if __name__ == "__main__":
    main()
