"""Fault tolerance of HBM collectives at world > 1 (direct transport; ranks share GPU 0).

Each iteration: a device Sum allreduce, a device Max allreduce, a device broadcast (pipelined
over 3 chunks), then an HBM checkpoint.  The mock engine kills ranks at given (rank, version, seqno, trial); the
survivors' barrier kernels give up (peer hang-up seen on the TCP plane), the communicator
epoch is rebuilt, and the restarted worker replays the missed results from the survivors'
HBM result logs.  The final model is checked against its closed form."""
import sys

import torch

import rabit_amd as rabit

rabit.init(sys.argv[1:], lib="mock", rabit_device=0, rabit_device_peer_buffer="1M",
           rabit_device_peer_timeout_sec=20)
rank, world = rabit.get_rank(), rabit.get_world_size()
dev = torch.device("cuda", 0)
N = (1 << 18) + 3
w = torch.zeros(N, device=dev, dtype=torch.float64)
version, meta = rabit.load_checkpoint_tensors({"w": w})
start = meta["next"] if version else 0
if version:
    print("[%d] resumed at version %d" % (rank, version), flush=True)
ITERS = 4
for it in range(start, ITERS):
    g = torch.full((N,), float(rank + it), device=dev, dtype=torch.float64)
    rabit.allreduce(g, rabit.SUM)
    m = torch.arange(5, device=dev, dtype=torch.int32) * (rank + 1) + it
    rabit.allreduce(m, rabit.MAX)
    assert torch.equal(m.cpu(), torch.arange(5, dtype=torch.int32) * world + it), m
    # 2.5 MiB with a 1 MiB stage: a pipelined broadcast of 3 chunks, so a kill at this op (seqno
    # 2) leaves the survivors mid-pipeline, and a restarted rank gets it back by replay
    b = torch.full(((5 << 19) + 777,), rank, device=dev, dtype=torch.uint8)
    rabit.broadcast_tensor(b, it % world)
    assert bool((b == it % world).all().item()), ("broadcast", it)
    w.add_(g)
    rabit.checkpoint_tensors({"w": w}, meta={"next": it + 1})
expect = float(sum(r + it for it in range(ITERS) for r in range(world)))
torch.cuda.synchronize()
assert torch.all(w == expect), (float(w[0]), expect)
st = rabit.stats()
assert st["device_direct"] == 1, st
rabit.finalize()
print("[%d] DEVFT OK replays=%d recovered=%d spilled=%d spilled_replays=%d"
      % (rank, st["n_device_replays"], st["n_recovered_ops"], st["n_spilled_results"],
         st["n_spilled_replays"]), flush=True)
