"""allreduce_graphable over the DIRECT transport, captured into a hipGraph and replayed, with
several ranks (they share the box's GPU, so RCCL is not up and the direct transport carries
every op).  The barriers inside the graph take their numbers from a device counter, so each
replay synchronises afresh with the peers' replays; eager collectives between replays use the
same counter.  Checked against closed forms after every replay:
  - a 3 MiB + odd fp32 sum (several stage chunks with a 1 MiB stage: parity flips inside the
    graph) and a small one (the one-shot form), plus a bf16 max;
  - the whole data-parallel step (forward, backward into buckets, bucket allreduce) as one graph,
    the replayed buckets equal to world x the local gradient."""
import sys

import numpy as np
import torch

import rabit_amd as rabit

rabit.init(sys.argv[1:], lib="base", rabit_device=0, rabit_device_peer_buffer="1M")
rank, world = rabit.get_rank(), rabit.get_world_size()
dev = torch.device("cuda", 0)
N = (3 << 20) // 4 + 77
x = torch.arange(N, device=dev, dtype=torch.float32).remainder_(97).add_(rank)
small = torch.full((1000,), float(rank + 1), device=dev)
y = torch.empty_like(x)
z = torch.empty_like(x)
h = torch.empty(4096, device=dev, dtype=torch.bfloat16)


def want_z(xv):
    # sum over ranks r of 2 * (base + r), base = x - rank on this rank
    base = xv - rank
    return 2.0 * (world * base + world * (world - 1) / 2.0) + 1.0


def step():
    torch.mul(x, 2.0, out=y)
    rabit.allreduce_graphable(y, rabit.SUM)
    torch.add(y, 1.0, out=z)
    small.fill_(float(rank + 1))
    rabit.allreduce_graphable(small, rabit.SUM)
    h.fill_(float(rank))
    rabit.allreduce_graphable(h, rabit.MAX)


side = torch.cuda.Stream()
side.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(side):
    step()  # eager: brings the transports up before any capture
torch.cuda.current_stream().wait_stream(side)
torch.cuda.synchronize()
assert torch.equal(z, want_z(x)), "eager"
st = rabit.stats()
assert st["device_direct"] == 1 and st["device_rccl"] == 0, st
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g, stream=side):
    step()
for i in range(5):
    x.add_(1.0)
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(z, want_z(x)), ("replay", i)
    assert bool((small == world * (world + 1) / 2).all().item()), ("small", i)
    assert bool((h.float() == world - 1).all().item()), ("max", i)
    # an eager collective between replays (same barrier counter)
    e = torch.full((5000,), float(rank), device=dev)
    rabit.allreduce(e, rabit.SUM)
    torch.cuda.synchronize()
    assert bool((e == world * (world - 1) / 2).all().item()), ("eager between", i)

from rabit_amd.parallel import GradientBuckets  # noqa: E402

torch.manual_seed(0)
model = torch.nn.Sequential(torch.nn.Linear(64, 64, bias=False), torch.nn.Tanh(),
                            torch.nn.Linear(64, 8, bias=False)).to(dev)
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
torch.cuda.synchronize()
g2 = torch.cuda.CUDAGraph()
with torch.cuda.graph(g2, stream=side):
    dp_step()
for b in buckets.buckets:
    b.zero_()
g2.replay()
torch.cuda.synchronize()
for p, gl in zip(model.parameters(), local):
    assert torch.allclose(p.grad, gl * world, rtol=1e-5, atol=1e-7), "replayed bucket != world x grad"
st = rabit.stats()
assert st["graph_direct_ops"] > 0, st
ok = rabit.allreduce(np.array([1], dtype=np.int32), rabit.SUM)[0] == world
assert ok
rabit.finalize()
print("[%d] GRAPHDIRECT OK graph_direct_ops=%d" % (rank, st["graph_direct_ops"]), flush=True)
