"""Run under torch.distributed.run: rabit rendezvous through the tracker in rank 0."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import rabit_amd as rabit  # noqa: E402
from rabit_amd.torchrun import init_from_env  # noqa: E402

ctx = init_from_env()
assert rabit.get_rank() == int(os.environ["RANK"]), "rabit rank must equal torchrun RANK"
x = torch.full((1 << 16,), float(ctx.rank + 1))
rabit.allreduce(x, rabit.SUM)
assert torch.all(x == ctx.world * (ctx.world + 1) / 2)
t = np.array([float(ctx.rank)])
assert rabit.allreduce(t, rabit.MAX)[0] == ctx.world - 1
for _ in range(3):
    rabit.allreduce(np.ones(4), rabit.SUM)
print("TORCHRUN OK rank=%d elided=%d" % (ctx.rank, rabit.stats()["n_consensus_elided"]), flush=True)
ctx.finalize()
