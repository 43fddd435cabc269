"""Pipelined direct broadcast, ranks sharing one GPU (launched per rank with RANK / WORLD_SIZE /
MASTER_* set, e.g. under rocprofv3 by tools/gpu_r3_s11.sh): 256 MiB broadcasts from root 0,
each checked, with the pipeline chunk given as argv[1] (0: automatic = 32 MiB, 8 chunks, 10
rounds, 9 barriers; 268435456: one chunk, the unpipelined structure of stage, scatter and
gather rounds); rank 0 prints one JSON line with the time and the broadcast counters."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import rabit_amd as rabit  # noqa: E402
from rabit_amd.torchrun import init_from_env  # noqa: E402


def main():
    nb = 256 << 20
    out = {}
    for chunk in sys.argv[1:2] or ["0"]:
        ctx = init_from_env(lib="standard", rabit_device=0, rabit_device_bcast_chunk=chunk)
        rank, world = rabit.get_rank(), rabit.get_world_size()
        dev = torch.device("cuda", 0)
        blob = torch.empty(nb, dtype=torch.uint8, device=dev)
        times = []
        for rep in range(6):
            blob.fill_(rep + 1 if rank == 0 else 0)
            torch.cuda.synchronize()
            rabit.allreduce(np.zeros(1, dtype=np.int32), rabit.SUM)
            t0 = time.perf_counter()
            rabit.broadcast_tensor(blob, 0)
            torch.cuda.synchronize()
            times.append(time.perf_counter() - t0)
            assert bool((blob[:: 1 << 16] == rep + 1).all().item()), ("broadcast", chunk, rep)
            rabit.checkpoint(None)
        st = rabit.stats()
        worst = float(rabit.allreduce(np.array([float(np.median(times[1:]))]), rabit.MAX)[0])
        out["auto" if chunk == "0" else "one_chunk"] = {
            "ms": round(worst * 1e3, 3), "direct_bcast_ops": st["direct_bcast_ops"],
            "direct_bcast_chunks": st["direct_bcast_chunks"]}
        del blob
        ctx.finalize()
    if int(os.environ.get("RANK", "0")) == 0:
        print(json.dumps({"probe": "bcast_pipeline", "bytes": nb,
                          "world": int(os.environ.get("WORLD_SIZE", "1")), "results": out}),
              flush=True)


if __name__ == "__main__":
    main()
