"""Per-op latency probe for small device allreduces (ranks share GPU 0): python-side time per
op in a tight loop vs the engine's own host time per op (stats t_allreduce)."""
import json
import sys
import time

import torch

import rabit_amd as rabit

lib = sys.argv[1] if len(sys.argv) > 1 else "base"
extra = dict(a.split("=", 1) for a in sys.argv[2:])
rabit.init([], lib=lib, rabit_device=0, **extra)
rank, world = rabit.get_rank(), rabit.get_world_size()
dev = torch.device("cuda", 0)
x = torch.ones(65536, device=dev)
for _ in range(20):
    rabit.allreduce(x, rabit.SUM)
torch.cuda.synchronize()
s0 = rabit.stats()
t0 = time.perf_counter()
N = 200
for _ in range(N):
    rabit.allreduce(x, rabit.SUM)
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / N
s1 = rabit.stats()
eng = (s1["t_allreduce"] - s0["t_allreduce"]) / N
if rank == 0:
    print(json.dumps({"lib": lib, "world": world, "extra": extra, "py_us_per_op": round(dt * 1e6, 1),
                      "engine_us_per_op": round(eng * 1e6, 1),
                      "direct": s1.get("device_direct"), "rccl": s1.get("device_rccl")}), flush=True)
rabit.finalize()
