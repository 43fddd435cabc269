"""rabit.link_probe() on ranks sharing the GPU: every value positive, the probe leaves the
transport usable (an allreduce after it is exact), and a second probe works too."""
import sys

import torch

import rabit_amd as rabit

rabit.init(sys.argv[1:], lib="standard", rabit_device=0, rabit_device_peer_buffer="32M")
rank, world = rabit.get_rank(), rabit.get_world_size()
dev = torch.device("cuda", 0)
x = torch.full((1 << 20,), float(rank + 1), device=dev)
rabit.allreduce(x, rabit.SUM)  # brings the transports up
for _ in range(2):
    lp = rabit.link_probe(8 << 20)
    assert lp is not None and set(lp) == set(rabit.core.LINK_PROBE_KEYS), lp
    assert all(v > 0 for v in lp.values()), lp
    x.fill_(float(rank + 1))
    rabit.allreduce(x, rabit.SUM)
    assert bool((x == world * (world + 1) / 2).all().item()), float(x[0])
if rank == 0:
    print("[0] link probe:", lp, flush=True)
rabit.finalize()
print("[%d] LINKPROBE OK" % rank, flush=True)
