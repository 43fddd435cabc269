"""prepare_fun must run for executed collectives and be skipped for replayed ones."""
import os
import sys

import numpy as np

import rabit_amd as rabit

rabit.init(sys.argv[1:], lib="mock")
rank, world = rabit.get_rank(), rabit.get_world_size()
attempt = int(os.environ.get("DMLC_NUM_ATTEMPT", "0"))
version, _ = rabit.load_checkpoint()
calls = []


def prepare(buf):
    calls.append(1)
    buf[:] = rank + np.arange(buf.size)


a = rabit.allreduce(np.zeros(4), rabit.MAX, prepare_fun=prepare)  # seq 0
assert np.array_equal(a, world - 1 + np.arange(4)), a
b = rabit.allreduce(np.ones(2), rabit.SUM)  # seq 1: the mock kill point
assert np.array_equal(b, world * np.ones(2))
if attempt > 0 and not calls:
    print("[%d] replayed-prepare-skipped" % rank, flush=True)
if attempt == 0:
    assert calls, "prepare must run when the collective executes"
rabit.checkpoint({"a": a})
rabit.finalize()
print("[%d] DONE" % rank, flush=True)
