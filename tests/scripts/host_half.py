"""16-bit floats on the host path: numpy float16 and torch bfloat16 CPU tensors, exact for
small integers (every reduction order gives the same value), tree and ring."""
import sys

import numpy as np
import torch

import rabit_amd as rabit

rabit.init(sys.argv[1:], lib="standard")
r, n = rabit.get_rank(), rabit.get_world_size()
for size in (1, 7, 1000, 100003):
    for op in (rabit.SUM, rabit.MAX, rabit.MIN):
        mine = ((np.arange(size) * (r + 3)) % 37).astype(np.float16)
        got = rabit.allreduce(mine, op)
        allv = np.stack([((np.arange(size) * (q + 3)) % 37).astype(np.float32) for q in range(n)])
        want = {rabit.SUM: allv.sum(0), rabit.MAX: allv.max(0),
                rabit.MIN: allv.min(0)}[op].astype(np.float16)
        assert got.dtype == np.float16 and np.array_equal(got, want), (size, op)
        t = torch.from_numpy(((np.arange(size) * (r + 3)) % 37).astype(np.float32)).to(torch.bfloat16)
        rabit.allreduce(t, op)
        want16 = torch.from_numpy(want.astype(np.float32)).to(torch.bfloat16)
        assert torch.equal(t, want16), (size, op, "bf16")
try:
    rabit.allreduce(np.ones(4, dtype=np.float16), rabit.BITOR)
    raise SystemExit("BITOR on float16 accepted")
except TypeError:
    pass
rabit.finalize()
print("[%d] H16 OK" % r, flush=True)
