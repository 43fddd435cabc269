"""Device (HBM) checkpoints under failure: the model lives in HBM, checkpoints are HBM
snapshots + pinned mirrors; a killed worker reloads its model from a survivor's lazy
snapshot.  Collectives use host arrays (TCP), so several workers can share one GPU."""
import sys

import numpy as np
import torch

import rabit_amd as rabit

rabit.init(sys.argv[1:], lib="mock", rabit_device=0)
rank, world = rabit.get_rank(), rabit.get_world_size()
dev = torch.device("cuda", 0)
w = torch.zeros(1 << 16, device=dev)
b = torch.zeros(7, dtype=torch.float64, device=dev)
version, meta = rabit.load_checkpoint_tensors({"w": w, "b": b})
if version == 0:
    w.fill_(1.0)
    b.fill_(0.5)
    start = 0
else:
    start = meta["next"]
    assert meta["tag"] == "xrabit", meta
    print("[%d] reloaded version %d from peers (device loads %d)"
          % (rank, version, rabit.stats()["n_device_ckpt_loads"]), flush=True)
for it in range(start, 4):
    g = rabit.allreduce(np.full(4, float(rank + it)), rabit.SUM)  # host plane
    expect = sum(r + it for r in range(world))
    assert np.all(g == expect)
    w.mul_(2.0).add_(float(g[0]))
    b.add_(1.0)
    rabit.checkpoint_tensors({"w": w, "b": b}, meta={"next": it + 1, "tag": "xrabit"})
# closed form of the model after 4 iterations
wv = 1.0
for it in range(4):
    wv = wv * 2.0 + sum(r + it for r in range(world))
torch.cuda.synchronize()
assert torch.all(w == wv), (float(w[0]), wv)
assert torch.all(b == 4.5)
st = rabit.stats()
rabit.finalize()
print("[%d] DEVCKPT OK slots=%d hbm=%d pinned=%d engine=%d"
      % (rank, st["ckpt_slots"], st["ckpt_hbm_bytes"], st["ckpt_pinned_bytes"],
         st["ckpt_mirror_engine"]), flush=True)
