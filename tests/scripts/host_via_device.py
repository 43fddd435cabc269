"""Large host (numpy) allreduces staged through HBM onto the device transports
(rabit_host_via_device=1); small ones stay on TCP.  Results are checked in closed form."""
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
after = rabit.stats()["n_device_ops"]
assert after - before == 2, (before, after)  # only the two large ones went to the device
rabit.finalize()
print("[%d] HOSTVIADEV OK" % rank, flush=True)
