"""allreduce_graphable inside a captured hipGraph (base engine, one GPU): the world-1 transport
hook gives the rank a one-rank RCCL communicator, so ncclAllReduce is called on the capturing
stream between the step's kernels (for one rank RCCL records it as a copy, not a reduction
kernel: this checks the API's capture and replay path).  Replays must give the eager result every time;
the fault-tolerant engines and BitOR must be refused.  argv[1]: base | standard."""
import sys

import torch

import rabit_amd as rabit

lib = sys.argv[1]
rabit.init(sys.argv[2:], lib=lib, rabit_device=0, rabit_world1_fastpath=0,
           rabit_device_world1_transport=1, rabit_device_algo="rccl")
dev = torch.device("cuda", 0)
x = torch.arange(1 << 20, device=dev, dtype=torch.float32).remainder_(113)
if lib != "base":
    try:
        rabit.allreduce_graphable(x, rabit.SUM)
    except RuntimeError as e:
        assert "fault tolerance" in str(e), e
        print("GRAPHAR REFUSED", flush=True)
    rabit.finalize()
    sys.exit(0)
try:
    rabit.allreduce_graphable(torch.zeros(8, device=dev, dtype=torch.int32), rabit.BITOR)
    raise AssertionError("BitOR accepted")
except RuntimeError as e:
    assert "not supported" in str(e), e

y = torch.empty_like(x)
z = torch.empty_like(x)
side = torch.cuda.Stream()


def step():
    torch.mul(x, 2.0, out=y)
    rabit.allreduce_graphable(y, rabit.SUM)
    torch.add(y, 1.0, out=z)
    for dt in (torch.bfloat16, torch.float16):  # extended dtypes ride through RCCL too
        h = y.to(dt)
        rabit.allreduce_graphable(h, rabit.MAX)
        z.add_(h.float()).sub_(y)


side.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(side):
    for _ in range(2):
        step()
torch.cuda.current_stream().wait_stream(side)
want = x * 2.0 + 1.0
torch.cuda.synchronize()
assert torch.equal(z, want), "eager"
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    step()
for i in range(4):
    x.add_(1.0)
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(z, x * 2.0 + 1.0), ("replay", i)
# the whole data-parallel step in one graph: forward, backward into the buckets, bucket allreduce
from rabit_amd.parallel import GradientBuckets  # noqa: E402

torch.manual_seed(0)
model = torch.nn.Sequential(torch.nn.Linear(64, 64, bias=False), torch.nn.Tanh(),
                            torch.nn.Linear(64, 8, bias=False)).to(dev)
# no averaging: the replayed buckets must hold world x the local gradient (every rank computes
# the same one from the same seed), which checks the reduction itself on a multi-GPU run; at
# world 1 RCCL records a copy and this is the identity
buckets = GradientBuckets(model.parameters(), bucket_mb=1.0, average=False)
xs = torch.randn(32, 64, device=dev)
local = torch.autograd.grad(model(xs).square().mean(), list(model.parameters()))


def dp_step():
    loss = model(xs).square().mean()
    buckets.backward(loss)
    buckets.reduce(graphable=True)
    return loss


with torch.cuda.stream(side):
    for _ in range(2):
        dp_step()
torch.cuda.current_stream().wait_stream(side)
eager = [b.clone() for b in buckets.buckets]
g2 = torch.cuda.CUDAGraph()
with torch.cuda.graph(g2):
    dp_step()
for b in buckets.buckets:
    b.zero_()
g2.replay()
torch.cuda.synchronize()
assert all(torch.equal(a, b) for a, b in zip(eager, buckets.buckets)), "graphed DP step"
world = rabit.get_world_size()
for p, g in zip(model.parameters(), local):
    assert torch.allclose(p.grad, g * world, rtol=1e-5, atol=1e-7), "replayed bucket != world x grad"
assert rabit.stats()["device_rccl"] == 1, "no RCCL communicator: nothing was captured"
print("GRAPHAR OK", flush=True)
rabit.finalize()
