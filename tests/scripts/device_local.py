"""Device-resident local (per-rank) checkpoints under failures (ranks share GPU 0 and talk
through the direct IPC transport; on an 8-GPU node the same calls run over RCCL/xGMI).

Each iteration: a device Sum allreduce of the global gradient, then a per-rank update of the
rank's own tensors (`loc`, `steps`: different sizes on every rank), then
checkpoint_tensors(global, local=...).  The robust engine keeps each rank's local tensors and
the replicas of its rabit_local_replica ring predecessors in HBM and replicates them with
device copies.  The mock engine kills ranks (`mock=rank,version,seq,trial`; seq 1 is the
checkpoint call); a restarted rank must get back its own local tensors bit for bit, which is
checked against their closed form right after the load and at the end."""
import os
import sys

import torch

import rabit_amd as rabit

ctx = None
params = dict(rabit_device=0, rabit_device_peer_buffer="1M", rabit_device_peer_timeout_sec=20)
if os.environ.get("XR_ENV_INIT") == "1":
    # ranks started one by one (e.g. each under its own profiler, tools/prof_local.sh)
    from rabit_amd.torchrun import init_from_env
    ctx = init_from_env(lib="mock", **params)
else:
    rabit.init(sys.argv[1:], lib="mock", **params)
rank, world = rabit.get_rank(), rabit.get_world_size()
dev = torch.device("cuda", 0)
N = (1 << 16) + 5
ITERS = 4


def local_expect(upto):
    """closed form of this rank's local tensors after `upto` iterations"""
    n = N + 97 * rank  # every rank's state has its own size
    v = float(sum(rank + 1 + it for it in range(upto)))
    loc = torch.full((n,), v, dtype=torch.float32)
    # a bit pattern that a misplaced or truncated copy cannot reproduce
    loc[::7] = -v - torch.arange(0, n, 7, dtype=torch.float32) % 1024
    steps = torch.tensor([upto, rank, n], dtype=torch.int64)
    return loc, steps


w = torch.zeros(N, device=dev, dtype=torch.float64)
loc0, steps0 = local_expect(0)
loc = loc0.to(dev)
steps = steps0.to(dev)
version, meta = rabit.load_checkpoint_tensors({"w": w}, local=[loc, steps])
start = meta["next"] if version else 0
if version:
    el, es = local_expect(start)
    assert torch.equal(loc.cpu(), el), "[%d] local tensor differs after the load" % rank
    assert torch.equal(steps.cpu(), es), (rank, steps.cpu(), es)
    print("[%d] resumed at version %d with its local tensors intact" % (rank, version), flush=True)
for it in range(start, ITERS):
    g = torch.full((N,), float(rank + it), device=dev, dtype=torch.float64)
    rabit.allreduce(g, rabit.SUM)
    w.add_(g)
    el, es = local_expect(it + 1)
    loc.copy_(el.to(dev))
    steps.copy_(es.to(dev))
    rabit.checkpoint_tensors({"w": w}, meta={"next": it + 1}, local=[loc, steps])
expect = float(sum(r + it for it in range(ITERS) for r in range(world)))
torch.cuda.synchronize()
assert torch.all(w == expect), (float(w[0]), expect)
el, es = local_expect(ITERS)
assert torch.equal(loc.cpu(), el) and torch.equal(steps.cpu(), es)
st = rabit.stats()
if ctx is not None:
    ctx.finalize()
else:
    rabit.finalize()
print("[%d] DEVLOCAL OK bytes_local_in=%d recovered=%d" %
      (rank, int(st["bytes_local_in"]), st["n_recovered_ops"]), flush=True)
