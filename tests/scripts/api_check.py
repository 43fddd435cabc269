"""Exercise the Python API on every rank and verify results in closed form."""
import sys

import numpy as np

import rabit_amd as rabit

lib = sys.argv[1] if len(sys.argv) > 1 else "standard"
rabit.init(sys.argv[2:], lib=lib)
rank, world = rabit.get_rank(), rabit.get_world_size()
assert rabit.is_distributed() or lib == "empty"
assert rabit.engine_name() in ("robust", "base", "mock", "empty")
# ---- allreduce: every dtype x op
for dt in [np.int8, np.uint8, np.int32, np.uint32, np.int64, np.uint64, np.float32, np.float64]:
    base = (np.arange(7) % 5).astype(dt)
    mine = (base + rank).astype(dt)
    s = rabit.allreduce(mine.copy(), rabit.SUM)
    assert np.array_equal(s, (base * world + world * (world - 1) // 2).astype(dt)), (dt, s)
    assert np.array_equal(rabit.allreduce(mine.copy(), rabit.MAX), (base + world - 1).astype(dt))
    assert np.array_equal(rabit.allreduce(mine.copy(), rabit.MIN), base)
    if np.dtype(dt).kind in "iu":
        bits = np.full(3, 1 << rank, dtype=dt)
        assert np.all(rabit.allreduce(bits, rabit.BITOR) == (1 << world) - 1)
# large enough to take the ring path (> 32K elements)
big = np.full(100003, float(rank + 1))
assert np.all(rabit.allreduce(big, rabit.SUM) == world * (world + 1) / 2)
# 2-d arrays come back flattened (reference behaviour)
m = rabit.allreduce(np.ones((2, 3)), rabit.SUM)
assert m.shape == (6,) and np.all(m == world)
# ---- broadcast of python objects from every root
for root in range(world):
    obj = {"root": root, "payload": list(range(root + 3))} if rank == root else None
    got = rabit.broadcast(obj, root)
    assert got == {"root": root, "payload": list(range(root + 3))}
# ---- allgather
g = rabit.allgather(np.array([rank, rank * 10], dtype=np.int64))
assert list(g) == [v for r in range(world) for v in (r, r * 10)]
# ---- checkpoint round trip
v, model = rabit.load_checkpoint()
assert v == 0 and model is None
rabit.checkpoint({"w": np.arange(3)})
assert rabit.version_number() == 1
rabit.lazy_checkpoint([1, 2, 3])
assert rabit.version_number() == 2
rabit.tracker_print("rank %d says hi" % rank)
assert len(rabit.get_processor_name()) > 0
st = rabit.stats()
assert (world == 1 or st["n_allreduce"] >= 30) and st["world_size"] == world
rabit.finalize()
print("[%d] API OK" % rank, flush=True)
