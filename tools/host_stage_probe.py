"""Host-buffer allreduce through HBM (rabit_host_via_device=1), ranks of one box: time a 128 MiB
float32 allreduce of a host tensor for the configuration given as engine parameters on the
command line (e.g. rabit_host_stage_chunk=16M rabit_host_stage_threads=4), and print the
stager's time split (host copies in / out, waits for a free input slot / for a chunk's result).

    python -m rabit_amd.launcher -n 2 -- python tools/host_stage_probe.py rabit_host_stage_chunk=8M
"""
import json
import sys
import time

import numpy as np
import torch

import rabit_amd as rabit


def main():
    args = [a for a in sys.argv[1:] if "=" in a]
    rabit.init(args, lib="standard", rabit_device=0, rabit_host_via_device=1)
    rank, world = rabit.get_rank(), rabit.get_world_size()
    n = (128 << 20) // 4
    x = torch.empty(n, dtype=torch.float32)
    x.fill_(1.0)
    rabit.allreduce(x, rabit.SUM)  # warm-up (transports, pinned slots, threads)
    assert float(x[0]) == world and float(x[-1]) == world
    times = []
    for _ in range(6):
        x.fill_(1.0)
        rabit.allreduce(np.zeros(1, dtype=np.int32), rabit.SUM)
        t0 = time.perf_counter()
        rabit.allreduce(x, rabit.SUM)
        times.append(time.perf_counter() - t0)
        assert float(x[n // 2]) == world
    med = float(np.median(times[1:]))
    worst = float(rabit.allreduce(np.array([med]), rabit.MAX)[0])
    st = rabit.stats()
    if rank == 0:
        print(json.dumps({"probe": "host_stage", "world": world, "args": args,
                          "ms": round(worst * 1e3, 2),
                          "speed_MiBps": round((128 << 20) / worst / 2 ** 20, 1),
                          "staged_ops": st["host_staged_ops"], "threads": st["host_stage_threads"],
                          "split": st["host_stage"]}), flush=True)
    rabit.finalize()


if __name__ == "__main__":
    main()
