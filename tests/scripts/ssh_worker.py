"""Worker of the launcher's --cluster ssh test: reports where it runs and checks an allreduce."""
import os

import numpy as np

import rabit_amd as rabit

rabit.init()
rank, world = rabit.get_rank(), rabit.get_world_size()
total = rabit.allreduce(np.array([rank + 1.0]), rabit.SUM)[0]
assert total == world * (world + 1) / 2, total
print("SSHW rank=%d host=%s local=%s/%s attempt=%s" % (
    rank, os.environ.get("FAKE_SSH_HOST"), os.environ.get("LOCAL_RANK"),
    os.environ.get("LOCAL_WORLD_SIZE"), os.environ.get("DMLC_NUM_ATTEMPT")), flush=True)
rabit.finalize()
