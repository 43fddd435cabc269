#!/usr/bin/env python3
"""Headline benchmark of xrabit on MI355X (BASELINE.json): 128 MB float32 Allreduce<Sum>.

Each timed step is one `rabit.allreduce(x, SUM)` of a 128 MB float32 HBM tensor through the
fault-tolerant (robust) engine: consensus bookkeeping, RCCL/xGMI allreduce written straight
into the HBM result log, and the copy back into the user tensor (the full per-op work a
rabit user pays; nothing is skipped).  At N=1 the engine's world-size-1 short-circuit is
disabled (rabit_world1_fastpath=0) so the step still runs the robust path on the device.

    python bench.py                       # N=1
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
        --master-port 29500 bench.py --gpus 8

Rank 0 prints one JSON line.  `value` is the whole-job aggregate throughput N * S / t
(GB/s, S = 128 MiB per rank, weak scaling); nccl-tests style `busbw_GBps` / `algbw_GBps` and
the per-step wall clock are reported alongside.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


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


def run_extras(rabit, torch, dev, world):
    """BASELINE.json configs 3 and 4 plus the checkpoint cost of config 5, on this job's ranks
    (result log and checkpoint paths included, as in the headline step)."""
    out = {}
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
    out["allreduce_128MiB_bf16_busbw_GBps"] = (round((128 << 20) / t / 1e9 * 2 * (world - 1) / world, 2)
                                               if world > 1 else None)
    rabit.checkpoint(None)
    del hb
    # config 5 (checkpoint part): HBM snapshot of a 256 MiB model every iteration
    model = torch.rand((256 << 20) // 4, dtype=torch.float32, device=dev)
    rabit.checkpoint_tensors({"w": model}, meta={"it": 0})
    # iterations longer than the async D2H mirror (~5 ms for 256 MiB) see only the snapshot
    t = _timed(rabit, torch, lambda: rabit.checkpoint_tensors({"w": model}, meta={"it": 1}), 5,
               settle=0.05, device_wide=False)
    out["checkpoint_256MiB_us"] = round(t * 1e6, 1)
    del model
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--size-mb", type=int, default=128)
    ap.add_argument("--engine", default="robust", choices=["robust", "base"])
    ap.add_argument("--check", type=int, default=1, help="verify one reduction first")
    ap.add_argument("--symmetric", type=int, default=-1,
                    help="allocate the buffer in rabit's symmetric heap (IPC-registered HBM that "
                         "the direct transport reads in place, like registered buffers in "
                         "nccl-tests); 0: a plain torch allocation (staged through a copy); "
                         "-1 (default): symmetric when N > 1 (at N=1 nothing is exchanged)")
    ap.add_argument("--extras", type=int, default=1,
                    help="after the timed loop, also time the other BASELINE configs: 1 GiB "
                         "broadcast, 64 MiB lazy (squared-gradient) allreduce fused vs unfused, "
                         "256 MiB HBM checkpoint")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("bench.py --gpus %d but WORLD_SIZE=%d: launch N>1 with "
                         "torch.distributed.run" % (args.gpus, world))
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
    # the rabit tracker lives in rank 0 next to the torchrun master port (rabit_amd.torchrun)
    n = args.size_mb * (1 << 20) // 4
    if args.symmetric < 0:
        args.symmetric = 1 if world > 1 else 0
    # + 48 MiB: the calibration's 32 MiB inputs come from the heap's free tail, so it times the
    # paths heap buffers take
    heap = {"rabit_device_symmetric_heap": str(n * 4 + (48 << 20))} if args.symmetric else {}
    ctx = init_from_env(lib="standard" if args.engine == "robust" else "base",
                        rabit_world1_fastpath=0, rabit_device=gpu, **heap)
    dev = torch.device("cuda", gpu)

    def barrier():
        rabit.allreduce(np.zeros(1, dtype=np.int32), rabit.SUM)

    if args.symmetric:
        x = rabit.symmetric_empty(n, torch.float32)
    else:
        x = torch.empty(n, dtype=torch.float32, device=dev)
    if args.check:
        x.fill_(float(rabit.get_rank() + 1))
        rabit.allreduce(x, rabit.SUM)
        expect = world * (world + 1) / 2.0
        ok = bool(torch.all(x == expect).item())
        bad = rabit.allreduce(np.array([0 if ok else 1], dtype=np.int32), rabit.SUM)[0]
        if bad:
            raise SystemExit("allreduce result check failed on %d rank(s)" % bad)
    g = torch.Generator(device=dev)
    g.manual_seed(1234 + rank)
    # |x| ~ 1e-3 keeps repeated in-place sums finite for hundreds of 8-rank steps
    x.copy_(torch.rand((n,), generator=g, dtype=torch.float32, device=dev).mul_(1e-3))

    for _ in range(args.warmup):
        rabit.allreduce(x, rabit.SUM)
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        rabit.allreduce(x, rabit.SUM)
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    elapsed = float(rabit.allreduce(np.array([elapsed]), rabit.MAX)[0])

    extras = run_extras(rabit, torch, dev, world) if args.extras else {}

    t_step = elapsed / args.steps
    size_bytes = n * 4
    algbw = size_bytes / t_step / 1e9
    busbw = algbw * (2.0 * (world - 1) / world) if world > 1 else 0.0
    aggregate = world * size_bytes / t_step / 1e9
    st = rabit.stats()
    rec = {
        "metric": "allreduce_128MB_fp32_sum_throughput",
        "value": round(aggregate, 2),
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
        "busbw_GBps": round(busbw, 2),
        "algbw_GBps": round(algbw, 2),
        "t_us": round(t_step * 1e6, 1),
        "value_definition": "N * bytes_per_rank / t_step (whole-job reduced bytes per second); "
                            "busbw = algbw * 2(N-1)/N as nccl-tests",
        "baseline_note": "reference publishes no numbers (BASELINE.md)",
        "consensus_elided": st.get("n_consensus_elided", 0),
        "device_epoch": st.get("device_epoch", 0),
        "transport": {"rccl": st.get("device_rccl", 0), "direct": st.get("device_direct", 0),
                      "zero_copy_chunks": st.get("zero_copy_chunks", 0),
                      "direct_min_bytes": st.get("device_direct_min", -1),
                      "calibration_us": st.get("calib_us"),
                      "direct_variant": "push" if st.get("direct_push") else "pull",
                      "calibration_push_us": st.get("calib_push_us"),
                      "calibration_heap_inputs": bool(st.get("calib_heap_src", 0))},
        "extras": extras,
        "reference_measured": reference_measured(world, aggregate),
    }
    if shared_gpu:
        rec["shared_gpu_rehearsal"] = "%d ranks on %d GPU(s): not an xGMI measurement" % (world, ngpu)
    if rank == 0:
        print(json.dumps(rec), flush=True)
    del x
    ctx.finalize()


if __name__ == "__main__":
    main()
