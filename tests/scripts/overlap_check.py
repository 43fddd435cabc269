"""Data-parallel MLP training with the bucket allreduces overlapped with backward
(CommThread + OverlappedBuckets) or run after it (GradientBuckets, same bucket layout).

    overlap_check.py MODE STEPS DEVICE [rabit params...]   MODE: seq | overlap, DEVICE: cpu | gpu

Prints the final-weight digest (identical on every rank and, for the same job, in both modes)
and the median step time.  Workers killed by mock kill points resume from the last checkpoint.
"""
import hashlib
import sys
import time

import numpy as np
import torch

import rabit_amd as rabit
from rabit_amd.parallel import GradientBuckets
from rabit_amd.parallel.overlap import CommThread, OverlappedBuckets

mode, steps, where = sys.argv[1], int(sys.argv[2]), sys.argv[3]
lib, params = "standard", []
for a in sys.argv[4:]:
    if a.startswith("lib="):
        lib = a[4:]
    else:
        params.append(a)
gpu = where == "gpu"
if not gpu:
    torch.set_num_threads(1)
dev = torch.device("cuda", 0) if gpu else torch.device("cpu")
extra = {"rabit_device": 0} if gpu else {}
comm = CommThread(lambda: rabit.init(params, lib=lib, **extra), device=0 if gpu else None)
call = comm.call
rank, world = call(rabit.get_rank), call(rabit.get_world_size)
torch.manual_seed(0)
hidden, layers = (1024, 8) if gpu else (128, 3)
mods = [torch.nn.Linear(64, hidden), torch.nn.Tanh()]
for _ in range(layers - 1):
    mods += [torch.nn.Linear(hidden, hidden), torch.nn.Tanh()]
model = torch.nn.Sequential(*mods, torch.nn.Linear(hidden, 1)).to(dev)
plist = list(model.parameters())
g = torch.Generator().manual_seed(100 + rank)
x = torch.randn(512, 64, generator=g).to(dev)
y = torch.randn(512, 1, generator=g).to(dev)
bucket_mb = 4.0 if gpu else 0.02
if mode == "overlap":
    buckets = OverlappedBuckets(plist, comm, bucket_mb=bucket_mb)
else:
    buckets = GradientBuckets(list(reversed(plist)), bucket_mb=bucket_mb)
flat = {"p%d" % i: p.data for i, p in enumerate(plist)}
version, state = call(rabit.load_checkpoint)
start = 0
if version > 0:
    start = state["next"]
    for k, v in flat.items():
        v.copy_(torch.from_numpy(state["w"][k]))
times = []
for step in range(start, steps):
    if gpu:
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    buckets.zero_grad()
    loss = torch.nn.functional.mse_loss(model(x), y)
    loss.backward()
    if mode == "overlap":
        buckets.finish()
    else:
        call(buckets.reduce)
    with torch.no_grad():
        for p in plist:
            p.add_(p.grad, alpha=-0.01)
    if gpu:
        torch.cuda.synchronize()
    times.append(time.perf_counter() - t0)
    if (step + 1) % 4 == 0:
        w = {k: v.detach().cpu().numpy().copy() for k, v in flat.items()}
        call(rabit.checkpoint, {"next": step + 1, "w": w})
digest = hashlib.sha1(b"".join(p.detach().cpu().numpy().tobytes() for p in plist)).hexdigest()[:16]
h = int(digest, 16) & ((1 << 62) - 1)
lo = call(rabit.allreduce, np.array([h], dtype=np.int64), rabit.MIN)[0]
hi = call(rabit.allreduce, np.array([h], dtype=np.int64), rabit.MAX)[0]
assert lo == hi, "ranks disagree on the weights"
med = float(np.median(times[2:] if len(times) > 4 else times)) if times else 0.0
comm.close()
print("[%d] OVERLAP OK mode=%s weights=%s step_us=%.1f" % (rank, mode, digest, med * 1e6),
      flush=True)
