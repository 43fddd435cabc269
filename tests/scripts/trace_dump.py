"""Record engine spans (rabit_trace=1) for a few collectives and dump a per-rank Chrome trace."""
import sys

import numpy as np

import rabit_amd as rabit

out_dir = sys.argv[1]
rabit.init(sys.argv[2:], rabit_trace=1)
r = rabit.get_rank()
for i in range(5):
    rabit.allreduce(np.full(1000, r + i, dtype=np.float32), rabit.SUM)
rabit.broadcast({"i": 1}, 0)
rabit.checkpoint({"w": 1})
n = rabit.dump_trace("%s/trace_%d.json" % (out_dir, r))
assert n > 0
rabit.finalize()
print("[%d] TRACE OK %d" % (r, n), flush=True)
