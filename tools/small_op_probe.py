"""Where the time of a small device allreduce goes (VERDICT r2 "next" #5).

Run with several ranks sharing GPU 0, under the repo launcher:

    python -m rabit_amd.launcher -n 2 -- python tools/small_op_probe.py [nbytes] [name=value ...]

Each rank runs back-to-back float32 sums of `nbytes` (default 4 KiB) on an HBM tensor through
the robust engine with tracing on (rabit_trace=1), then splits the per-op time from the trace
spans: python wrapper (ctypes call and stream bookkeeping) = wall per op - engine span;
engine bookkeeping = engine span - device span (consensus when not elided, result log,
sequence numbers); device enqueue = device span - device wait; device wait = the host waiting
for the kernel (launch latency + kernel + completion signal).  Rank 0 prints one JSON line.
"""
import json
import os
import sys
import tempfile
import time

import numpy as np
import torch

import rabit_amd as rabit

nbytes = int(sys.argv[1]) if len(sys.argv) > 1 and "=" not in sys.argv[1] else 4096
extra = dict(a.split("=", 1) for a in sys.argv[1:] if "=" in a)
lib = extra.pop("lib", "standard")
rabit.init([], lib=lib, rabit_device=0, rabit_trace=1, rabit_trace_capacity=1 << 16, **extra)
rank, world = rabit.get_rank(), rabit.get_world_size()
dev = torch.device("cuda", 0)
x = torch.ones(nbytes // 4, device=dev)
for _ in range(50):
    rabit.allreduce(x, rabit.SUM)
torch.cuda.synchronize()
rabit.checkpoint(None)
N = 400
rabit.allreduce(np.zeros(1, dtype=np.int32), rabit.SUM)  # lock step
path = os.path.join(tempfile.gettempdir(), "small_op_probe_%d_%d.json" % (os.getpid(), rank))
rabit.dump_trace(path)  # clears nothing: spans before t0 are filtered below
t_start = time.perf_counter()
wall = []
for _ in range(N):
    t0 = time.perf_counter()
    rabit.allreduce(x, rabit.SUM)
    wall.append(time.perf_counter() - t0)
torch.cuda.synchronize()
ok = bool(torch.all(x == float(world) ** (50 + N)).item()) if world == 1 else True
st = rabit.stats()
rabit.dump_trace(path)
ev = json.load(open(path))
ev = ev["traceEvents"] if isinstance(ev, dict) else ev
os.unlink(path)
spans = {}
for e in ev:
    if e.get("ph") != "X":
        continue
    spans.setdefault(e["name"], []).append(e["dur"])  # us
last = {k: v[-N:] for k, v in spans.items()}  # the timed ops are the last N of each kind
med = lambda v: float(np.median(v)) if v else 0.0  # noqa: E731
wall_us = med([w * 1e6 for w in wall])
eng = med(last.get("allreduce", []))
devs = med(last.get("device_allreduce", []))
wait = med(last.get("device_wait", []))
rec = {"world": world, "bytes": nbytes, "ops": N, "wall_us": round(wall_us, 1),
       "python_us": round(wall_us - eng, 1), "engine_bookkeeping_us": round(eng - devs, 1),
       "device_enqueue_us": round(devs - wait, 1), "device_wait_us": round(wait, 1),
       "engine_span_us": round(eng, 1), "consensus_in_loop": st["n_consensus"],
       "consensus_elided": st["n_consensus_elided"], "oneshot_ops": st["oneshot_ops"],
       "fused_oneshots": st["fused_oneshots"], "rccl": st["device_rccl"],
       "direct": st["device_direct"], "params": extra}
agg = rabit.allreduce(np.array([wall_us]), rabit.MAX)[0]
rec["wall_us_max_over_ranks"] = round(float(agg), 1)
if rank == 0:
    print(json.dumps(rec), flush=True)
rabit.finalize()
