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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--size-mb", type=int, default=128)
    ap.add_argument("--engine", default="robust", choices=["robust", "base"])
    ap.add_argument("--check", type=int, default=1, help="verify one reduction first")
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

    torch.cuda.set_device(local_rank)
    # the rabit tracker lives in rank 0 next to the torchrun master port (rabit_amd.torchrun)
    ctx = init_from_env(lib="standard" if args.engine == "robust" else "base",
                        rabit_world1_fastpath=0)
    dev = torch.device("cuda", local_rank)

    def barrier():
        rabit.allreduce(np.zeros(1, dtype=np.int32), rabit.SUM)

    n = args.size_mb * (1 << 20) // 4
    if args.check:
        y = torch.full((n,), float(rabit.get_rank() + 1), dtype=torch.float32, device=dev)
        rabit.allreduce(y, rabit.SUM)
        expect = world * (world + 1) / 2.0
        ok = bool(torch.all(y == expect).item())
        bad = rabit.allreduce(np.array([0 if ok else 1], dtype=np.int32), rabit.SUM)[0]
        if bad:
            raise SystemExit("allreduce result check failed on %d rank(s)" % bad)
        del y
    g = torch.Generator(device=dev)
    g.manual_seed(1234 + rank)
    # |x| ~ 1e-3 keeps repeated in-place sums finite for hundreds of 8-rank steps
    x = torch.rand((n,), generator=g, dtype=torch.float32, device=dev).mul_(1e-3)

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
                   "engine": args.engine, "size_bytes_per_rank": size_bytes},
        "busbw_GBps": round(busbw, 2),
        "algbw_GBps": round(algbw, 2),
        "t_us": round(t_step * 1e6, 1),
        "value_definition": "N * bytes_per_rank / t_step (whole-job reduced bytes per second); "
                            "busbw = algbw * 2(N-1)/N as nccl-tests",
        "baseline_note": "reference publishes no numbers (BASELINE.md)",
        "consensus_elided": st.get("n_consensus_elided", 0),
        "device_epoch": st.get("device_epoch", 0),
    }
    if rank == 0:
        print(json.dumps(rec), flush=True)
    del x
    ctx.finalize()


if __name__ == "__main__":
    main()
