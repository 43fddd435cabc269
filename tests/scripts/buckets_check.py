"""GradientBuckets over HBM (direct transport, ranks share GPU 0), plain and symmetric-heap
buckets: after backward + reduce every rank holds the average of the per-rank gradients."""
import sys

import torch

import rabit_amd as rabit
from rabit_amd.parallel.data_parallel import GradientBuckets

sym = sys.argv[1] == "1"
# two-shot for every bucket (one-shot ops never read their input in place), so the symmetric
# buckets exercise the zero-copy path
rabit.init(sys.argv[2:], lib="standard", rabit_device=0, rabit_device_oneshot_max=0,
           **({"rabit_device_symmetric_heap": "64M"} if sym else {}))
rank, world = rabit.get_rank(), rabit.get_world_size()
dev = torch.device("cuda", 0)
torch.manual_seed(0)
model = torch.nn.Sequential(torch.nn.Linear(64, 256), torch.nn.ReLU(), torch.nn.Linear(256, 8))
model = model.to(dev)
buckets = GradientBuckets(model.parameters(), bucket_mb=0.05, symmetric=sym)
assert len(buckets.buckets) >= 2
g = torch.Generator(device="cpu").manual_seed(100 + rank)
x = torch.randn(32, 64, generator=g).to(dev)
for it in range(3):
    buckets.zero_grad()
    model(x).pow(2).mean().backward()
    local = [p.grad.detach().clone() for p in model.parameters()]
    buckets.reduce()
    # reference: average of every rank's local gradient, gathered through the host plane
    for p, lg in zip(model.parameters(), local):
        tot = rabit.allreduce(lg.cpu().double().numpy().ravel(), rabit.SUM)
        want = torch.as_tensor(tot).view_as(lg) / world
        assert torch.allclose(p.grad.double().cpu(), want, rtol=1e-5, atol=1e-6), it
st = rabit.stats()
if sym and world > 1:
    assert st["zero_copy_chunks"] > 0, st
rabit.finalize()
print("[%d] BUCKETS OK sym=%d" % (rank, sym), flush=True)
