"""Direct (IPC peer-memory) transport sweep with per-phase timing.

Run on one GPU box with several ranks sharing its GPU:

    python -m rabit_amd.launcher -n 4 python tools/direct_bench.py

All "remote" reads are then local HBM reads, so the numbers bound the transport's fixed costs
(launches, flag barriers, stage copy) and the HBM-side cost of each phase; the xGMI-bound
phases of an 8-GPU run (reduce, gather) are not represented.  Rank 0 prints one JSON line per
size with the median op time and the average hipEvent time of each phase.
"""
import json
import os
import sys
import time

import numpy as np
import torch

import rabit_amd as rabit


def main():
    sym = os.environ.get("XR_SYM", "0") == "1"
    fused = os.environ.get("XR_FUSED", "1")
    timing = os.environ.get("XR_PHASE", "0")
    rabit.init(sys.argv[1:], lib=os.environ.get("XR_LIB", "base"), rabit_device=0, rabit_device_phase_timing=timing,
               rabit_device_algo="direct", rabit_device_fused=fused,
               **({"rabit_device_symmetric_heap": "160M"} if sym else {}))
    rank, world = rabit.get_rank(), rabit.get_world_size()
    dev = torch.device("cuda", 0)
    sizes = (256 << 10, 1 << 20, 4 << 20, 16 << 20, 32 << 20, 128 << 20)
    if sym:
        sizes = (1 << 20, 8 << 20, 128 << 20)  # bump-allocated heap: keep the total small
    if os.environ.get("XR_SIZES"):
        sizes = tuple(int(v) for v in os.environ["XR_SIZES"].split(","))
    reps = int(os.environ.get("XR_REPS", "10"))
    for nbytes in sizes:
        if sym:
            x = rabit.symmetric_empty(nbytes // 4)
            x.fill_(1.0)
        else:
            x = torch.ones(nbytes // 4, device=dev)
        for _ in range(3):
            rabit.allreduce(x, rabit.SUM)
        times = []
        before = rabit.stats()
        for _ in range(reps):
            torch.cuda.synchronize()
            rabit.allreduce(np.zeros(1, dtype=np.int32), rabit.SUM)  # host barrier
            t0 = time.perf_counter()
            rabit.allreduce(x, rabit.SUM)
            torch.cuda.synchronize()
            times.append(time.perf_counter() - t0)
        st = rabit.stats()
        phase = {}
        n0, n1 = before.get("direct_timed_ops", 0), st.get("direct_timed_ops", 0)
        if n1 > n0:
            p0 = before.get("direct_phase_us") or {}
            for k, v in st["direct_phase_us"].items():
                phase[k] = round((v * n1 - p0.get(k, 0.0) * n0) / (n1 - n0), 1)
        med = float(np.median(times))
        med = float(rabit.allreduce(np.array([med]), rabit.MAX)[0])
        if rank == 0:
            print(json.dumps({
                "world_on_one_gpu": world, "bytes": nbytes, "symmetric": sym, "t_us": round(med * 1e6, 1),
                "fused": fused == "1", "fused_chunks": st.get("fused_chunks", 0),
                "fused_oneshots": st.get("fused_oneshots", 0),
                "direct_push": st.get("direct_push", 0),
                "direct_pipeline": st.get("direct_pipeline", 0),
                "pipelined_ops": st.get("pipelined_ops", 0),
                "phase_us": phase, "timed_ops": n1 - n0,
            }), flush=True)
        del x
    rabit.finalize()


if __name__ == "__main__":
    main()
