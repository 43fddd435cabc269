"""Fused lazy prepare on the RCCL path (VERDICT r2 "next" #8), one GPU.

World 1 with device ops routed through a one-rank RCCL communicator
(rabit_device_world1_transport=1, rabit_device_algo=rccl).  A squared-gradient allreduce
(allreduce_prepared, PREP_SQUARE) of 64 MiB float32 takes the kernel-reduced RCCL path, whose
reduce kernel squares each source as it loads it: under rocprofv3 --kernel-trace no
PrepareTileKernel runs.  Prints one JSON line: median op time and the result check.
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import rabit_amd as rabit  # noqa: E402
from rabit_amd.tracker import RabitTracker  # noqa: E402

tracker = RabitTracker("127.0.0.1", 1, port=9481, print_fn=lambda m: None).start(1)
rabit.init(sys.argv[1:], lib="standard", rabit_tracker_uri="127.0.0.1",
           rabit_tracker_port=tracker.port, rabit_task_id=0, rabit_world_size=1,
           rabit_world1_fastpath=0, rabit_device_world1_transport=1, rabit_device_algo="rccl",
           rabit_device=0)
dev = torch.device("cuda", 0)
n = (64 << 20) // 4
g = torch.rand(n, device=dev)
acc = torch.empty_like(g)
want = g * g
times = []
for i in range(12):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    rabit.allreduce_prepared(acc, g, rabit.SUM, rabit.PREP_SQUARE)
    torch.cuda.synchronize()
    if i >= 2:
        times.append(time.perf_counter() - t0)
    rabit.checkpoint(None)
ok = bool(torch.equal(acc, want))
times.sort()
st = rabit.stats()
print(json.dumps({"bytes": n * 4, "median_us": round(times[len(times) // 2] * 1e6, 1),
                  "result_ok": ok, "rccl": st["device_rccl"], "n_device_ops": st["n_device_ops"]}),
      flush=True)
rabit.finalize()
tracker.join(30)
sys.exit(0 if ok else 1)
