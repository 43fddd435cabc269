"""Per-op time of base-engine allreduces over the direct transport: eager calls against the same
ops captured into one hipGraph (allreduce_graphable) and replayed.  Ranks share the box's GPU
(launcher); rank 0 prints one JSON line per size.

    python -m rabit_amd.launcher -n 2 -- python tools/graph_direct_bench.py
"""
import json
import os
import sys
import time

import numpy as np
import torch

import rabit_amd as rabit


def main():
    rabit.init(sys.argv[1:], lib="base", rabit_device=0)
    rank, world = rabit.get_rank(), rabit.get_world_size()
    dev = torch.device("cuda", 0)
    side = torch.cuda.Stream()
    sizes = (4096, 1 << 20, 16 << 20)
    if os.environ.get("XR_SIZES"):
        sizes = tuple(int(v) for v in os.environ["XR_SIZES"].split(","))
    for nbytes in sizes:
        x = torch.full((nbytes // 4,), float(rank + 1), device=dev)
        ops = 64 if nbytes <= (1 << 20) else 16
        # eager (host waits for each op)
        rabit.allreduce(x, rabit.SUM)
        torch.cuda.synchronize()
        rabit.allreduce(np.zeros(1, dtype=np.int32), rabit.SUM)
        t0 = time.perf_counter()
        for _ in range(ops):
            rabit.allreduce(x, rabit.SUM)
        torch.cuda.synchronize()
        eager = (time.perf_counter() - t0) / ops
        # graph: the same ops captured once, replayed
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            rabit.allreduce_graphable(x, rabit.SUM)
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=side):
            for _ in range(ops):
                x.fill_(float(rank + 1))
                rabit.allreduce_graphable(x, rabit.SUM)
        g.replay()
        torch.cuda.synchronize()
        assert bool((x == world * (world + 1) / 2).all().item())
        rabit.allreduce(np.zeros(1, dtype=np.int32), rabit.SUM)
        reps = 3
        t0 = time.perf_counter()
        for _ in range(reps):
            g.replay()
        torch.cuda.synchronize()
        graphed = (time.perf_counter() - t0) / (reps * ops)
        e = float(rabit.allreduce(np.array([eager]), rabit.MAX)[0])
        gr = float(rabit.allreduce(np.array([graphed]), rabit.MAX)[0])
        if rank == 0:
            print(json.dumps({"world_on_one_gpu": world, "bytes": nbytes, "ops": ops,
                              "eager_us": round(e * 1e6, 1), "graphed_us": round(gr * 1e6, 1),
                              "graphed_includes": "a fill kernel per op"}), flush=True)
        del g
    rabit.finalize()


if __name__ == "__main__":
    main()
