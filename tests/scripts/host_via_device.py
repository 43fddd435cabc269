"""Large host (numpy) allreduces staged through HBM onto the device transports
(rabit_host_via_device=1); small ones stay on TCP.  Results are checked in closed form.  With
rabit_host_stage_chunk=1M (given by the test) ops of 2 MiB and more can go through the pipelined stager
(H2D, device allreduce and D2H of consecutive chunks overlap, the last chunk short):
rabit_host_stage=1 always, =auto after timing one op of each form, =0 never."""
import sys

import numpy as np

import rabit_amd as rabit

rabit.init(sys.argv[1:], lib="standard", rabit_device=0, rabit_host_via_device=1,
           rabit_host_via_device_min="64K")
rank, world = rabit.get_rank(), rabit.get_world_size()
before = rabit.stats()["n_device_ops"]
for n in (10, (3 << 20) // 8 + 1):
    a = np.arange(n, dtype=np.float64) + rank
    got = rabit.allreduce(a, rabit.SUM)
    assert np.array_equal(got, np.arange(n) * world + world * (world - 1) / 2), n
    b = (np.arange(n, dtype=np.int32) % 7) * (rank + 1)
    got = rabit.allreduce(b, rabit.MAX)
    assert np.array_equal(got, (np.arange(n) % 7) * world), n
# pipelined sizes: a whole number of chunks, a short tail, odd element counts; sum and max
for n in ((4 << 20) // 4, (5 << 20) // 8 + 3, (9 << 20) // 4 + 17):
    dt = np.float32 if n % 2 == 0 else np.float64
    a = (np.arange(n) % 1000).astype(dt) + rank
    got = rabit.allreduce(a, rabit.SUM)
    assert np.array_equal(got, ((np.arange(n) % 1000) * world + world * (world - 1) / 2).astype(dt)), n
    b = ((np.arange(n, dtype=np.int64) * 7 + rank * 13) % 1001).astype(np.int32)
    got = rabit.allreduce(b, rabit.MAX)
    want = np.max(np.stack([((np.arange(n, dtype=np.int64) * 7 + r * 13) % 1001) for r in range(world)]), 0)
    assert np.array_equal(got, want.astype(np.int32)), n
st = rabit.stats()
after = st["n_device_ops"]
assert after - before == 8, (before, after)  # only the large ones went to the device
# with 1 MiB chunks every op of 2 MiB or more is eligible for the pipeline: the 3 MiB float64
# sum above and the 6 below (the 1.5 MiB int32 max above is staged whole)
argv = sys.argv[1:]
if "rabit_host_stage=1" in argv:
    assert st["host_staged_ops"] == 7 and st["host_stage_choice"] == "pipelined", st
    assert st["host_stage_threads"] >= 1, st
elif "rabit_host_stage=auto" in argv:
    # a warm-up op and a timed op whole, a timed op pipelined, then one form kept everywhere
    assert st["host_stage_choice"] in ("pipelined", "whole"), st
    assert all(r > 0 for r in st["host_stage_rates_GBps"]), st
    want = 5 if st["host_stage_choice"] == "pipelined" else 1
    assert st["host_staged_ops"] == want, st
    choice = rabit.allreduce(np.array([st["host_stage_choice"] == "pipelined"], dtype=np.int32),
                             rabit.SUM)[0]
    assert choice in (0, world), choice
else:
    assert st["host_staged_ops"] == 0, st
rabit.finalize()
print("[%d] HOSTVIADEV OK" % rank, flush=True)
