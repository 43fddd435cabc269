"""Runs of small broadcasts while a tree leaf dies, with results kept on only some ranks.

With 10 ranks and rabit_global_replica=5 the retention round is 2: each result stays on the 5
ranks whose rank % 2 equals its seqno % 2.  Small broadcasts to a dead leaf can "succeed" into
kernel socket buffers, so with consensus elision (the default) the survivors may run several
sequence numbers past the failure before a link error stops them; the restarted leaf and any
laggards must then be served from the ranks that kept each result.  Every broadcast and
allreduce result is checked against its closed form on every rank.
"""
import sys

import numpy as np

import rabit_amd as rabit

rabit.init(sys.argv[1:], lib="mock")
rank, world = rabit.get_rank(), rabit.get_world_size()
version, model = rabit.load_checkpoint()
if version == 0:
    model = {"acc": 0}
NVER, NBCAST = 4, 24
for v in range(version, NVER):
    for i in range(NBCAST):
        root = (v * 7 + i) % world
        got = rabit.broadcast((v, i, root * 1000 + i) if rank == root else None, root)
        assert got == (v, i, root * 1000 + i), (rank, v, i, got)
        if i % 8 == 7:
            s = rabit.allreduce(np.array([rank + v + i], dtype=np.int64), rabit.SUM)
            assert int(s[0]) == world * (v + i) + world * (world - 1) // 2, (rank, v, i, s)
            model["acc"] += int(s[0])
    rabit.checkpoint(model)
expect = sum(world * (v + i) + world * (world - 1) // 2
             for v in range(NVER) for i in range(NBCAST) if i % 8 == 7)
assert model["acc"] == expect, (model, expect)
st = rabit.stats()
rabit.finalize()
print("[%d] BCAST-LEAF OK elided=%d recovered=%d" % (rank, st["n_consensus_elided"],
                                                     st["n_recovered_ops"]), flush=True)
