"""Back-to-back small HBM allreduces through the direct transport, every result checked: the
stage buffers alternate by parity and a rank's next op on the same parity overwrites its stage,
so a protocol that let a fast rank overwrite data a slow peer still reads would show up here as
a wrong sum.  Sizes cycle through the fused one-shot (<= 64 KiB), the classic one-shot and the
two-shot path; values change every op.  argv: [ops] then engine parameters."""
import sys

import numpy as np
import torch

import rabit_amd as rabit

nops = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 2000
params = [a for a in sys.argv[1:] if "=" in a]
rabit.init(params, lib="standard", rabit_device=0, rabit_device_peer_buffer="1M",
           rabit_device_peer_timeout_sec=20)
rank, world = rabit.get_rank(), rabit.get_world_size()
dev = torch.device("cuda", 0)
sizes = [1, 3, 256, 1000, 4096, 16384 + 5, 65536 // 4, 100000 // 4, 262144 // 4, (1 << 20) // 4]
bufs = {n: torch.empty(n, dtype=torch.float32, device=dev) for n in sizes}
base = {n: torch.arange(n, dtype=torch.float32, device=dev).remainder_(97) for n in sizes}
want = {n: torch.arange(n, dtype=torch.float64).remainder_(97) for n in sizes}
bad = 0
for k in range(nops):
    n = sizes[k % len(sizes)]
    # value of rank r at op k: (i % 97) + 3 r + k: exact in fp32 for these magnitudes
    x = bufs[n]
    torch.add(base[n], float(3 * rank + k), out=x)
    rabit.allreduce(x, rabit.SUM)
    if k % 7 == 0 or k >= nops - len(sizes):
        exp = want[n] * world + 3 * world * (world - 1) / 2 + k * world
        if not torch.equal(x.cpu().double(), exp):
            bad += 1
            print("[%d] op %d (n=%d) wrong" % (rank, k, n), flush=True)
    else:
        # no host read in between: the next op is enqueued right behind this one
        pass
    if k % 500 == 499:
        rabit.checkpoint(None)  # bounded result log
torch.cuda.synchronize()
st = rabit.stats()
bad = int(rabit.allreduce(np.array([bad], dtype=np.int64), rabit.SUM)[0])
assert bad == 0, bad
assert st["oneshot_ops"] > 0, st
rabit.finalize()
print("[%d] STRESS OK ops=%d fused_oneshots=%d oneshot=%d" % (rank, nops, st["fused_oneshots"],
                                                            st["oneshot_ops"]), flush=True)
