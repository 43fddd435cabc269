"""A prepare function that never returns on the first attempt of one rank.

With rabit_hang_timeout_sec the stuck rank leaves with a restartable status; its peers, which
only wait for it, see the links drop and recover, and the restarted rank replays the results it
missed and runs the stuck collective again.  Without it the job would hang forever (the
reference cannot detect this case: every rank is blocked, none has failed).
"""
import os
import sys
import time

import numpy as np

import rabit_amd as rabit

HANG_RANK = 2
rabit.init(sys.argv[1:], lib="standard")
rank, world = rabit.get_rank(), rabit.get_world_size()
attempt = int(os.environ.get("DMLC_NUM_ATTEMPT", "0"))
version, model = rabit.load_checkpoint()
if version == 0:
    model = {"w": np.zeros(4)}
for it in range(version, 3):
    g = rabit.allreduce(np.full(4, rank + 1.0), rabit.SUM)  # seq 0
    assert np.array_equal(g, np.full(4, world * (world + 1) / 2.0)), g

    def prepare(buf, it=it):
        if it == 1 and rank == HANG_RANK and attempt == 0:
            print("[%d] prepare stuck" % rank, flush=True)
            time.sleep(3600)
        buf[:] = rank + it

    m = rabit.allreduce(np.zeros(4), rabit.MAX, prepare_fun=prepare)  # seq 1
    assert np.array_equal(m, np.full(4, world - 1.0 + it)), m
    model["w"] += g + m
    rabit.checkpoint(model)
want = sum(np.full(4, world * (world + 1) / 2.0) + world - 1.0 + it for it in range(3))
assert np.array_equal(model["w"], want), model["w"]
rabit.finalize()
print("[%d] DONE attempt=%d" % (rank, attempt), flush=True)
