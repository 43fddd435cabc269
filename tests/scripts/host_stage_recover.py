"""A rank killed and restarted while host-buffer allreduces are staged through HBM with
rabit_host_stage=auto.  The survivors have finished the staging trial (warm-up,
a whole op, a pipelined op, then an agreed choice) before the kill; the restarted rank starts
with a fresh process.  The trial state is per epoch and restarts on every rank when the device
transports come back up, so all ranks keep running the same form and the same nested host
allreduce of the trial's rates.  Each iteration: 3 staged allreduces (3 MiB float32, 1 MiB
chunks), then a checkpoint of the running model; checked against the closed form."""
import sys

import numpy as np

import rabit_amd as rabit

rabit.init(sys.argv[1:], lib="mock", rabit_device=0, rabit_host_via_device=1,
           rabit_host_via_device_min="64K", rabit_host_stage="auto",
           rabit_host_stage_chunk="1M", rabit_device_peer_timeout_sec=20)
rank, world = rabit.get_rank(), rabit.get_world_size()
N = (3 << 20) // 4
version, model = rabit.load_checkpoint()
if version == 0:
    model = np.zeros(N, dtype=np.float32)
else:
    print("[%d] resumed at version %d" % (rank, version), flush=True)
ITERS = 5
for it in range(version, ITERS):
    for k in range(3):
        a = (np.arange(N) % 97).astype(np.float32) + rank + k + it
        got = rabit.allreduce(a, rabit.SUM)
        want = ((np.arange(N) % 97) + k + it) * world + world * (world - 1) / 2
        assert np.array_equal(got, want.astype(np.float32)), (it, k)
        model += got
    rabit.checkpoint(model)
want = np.zeros(N, dtype=np.float64)
for it in range(ITERS):
    for k in range(3):
        want += ((np.arange(N) % 97) + k + it) * world + world * (world - 1) / 2
assert np.array_equal(model, want.astype(np.float32)), "model"
st = rabit.stats()
rabit.finalize()
print("[%d] HOSTSTAGE RECOVER OK choice=%s staged=%d" % (rank, st["host_stage_choice"],
                                                         st["host_staged_ops"]), flush=True)
