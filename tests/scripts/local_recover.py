"""Pickled global + local checkpoints under mock failures (the reference's
test/local_recover.py scenario), with the result verified in closed form."""
import sys

import numpy as np

import rabit_amd as rabit

rabit.init(sys.argv[1:], lib="mock")
rank, world = rabit.get_rank(), rabit.get_world_size()
n, nround = 10, 3
data = np.ones(n) * rank
version, model, local = rabit.load_checkpoint(True)
if version == 0:
    model, local = np.zeros(n), np.ones(n)
else:
    print("[%d] restart from version %d" % (rank, version), flush=True)
for i in range(version, nround):
    # local is identical on every rank here, so the sum has a closed form
    expect = world * (world - 1) / 2.0 + world * model + world * local
    res = rabit.allreduce(data + model + local, rabit.SUM)
    assert np.allclose(res, expect), (rank, i, res, expect)
    model = res
    local[:] = i
    rabit.checkpoint(model, local)
rabit.finalize()
print("[%d] DONE" % rank, flush=True)
