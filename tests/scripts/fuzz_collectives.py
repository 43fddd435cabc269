"""Randomised collectives on CPU ranks, checked exactly against numpy.

    fuzz_collectives.py SEED NCASE [rabit params...]

Every rank draws the same sequence of cases from SEED (kind, size, dtype, op, root, slices) and
regenerates every rank's input from (SEED, case, rank), so it can compute the expected result
of each collective on its own.  Sizes cover 0, 1, odd lengths, buffer-size boundaries and sizes
larger than the ring / shared-memory stage buffers the parameters set; allgather slices have
random, possibly empty, sizes and a random start, so they wrap around the end of the buffer.
Integer-valued inputs keep float sums exact in any reduction order.
"""
import ctypes
import sys

import numpy as np

import rabit_amd as rabit
from rabit_amd import core

seed, ncase = int(sys.argv[1]), int(sys.argv[2])
lib = "standard"
params = []
for a in sys.argv[3:]:
    if a.startswith("lib="):
        lib = a[4:]
    else:
        params.append(a)
rabit.init(params, lib=lib)
rank, world = rabit.get_rank(), rabit.get_world_size()
DTYPES = [np.int8, np.uint8, np.int32, np.uint32, np.int64, np.uint64, np.float32, np.float64]
SIZES = [0, 1, 2, 3, 7, 31, 255, 1000, 1023, 4097, 40000, 65537, 300001]
OPS = [rabit.MAX, rabit.MIN, rabit.SUM, rabit.BITOR]


def draw_cases():
    """the whole case list, identical on every rank (a restarted rank skips the done ones)"""
    rng = np.random.default_rng(seed)
    cases = []
    for _ in range(ncase):
        kind = int(rng.integers(0, 3))
        size = int(rng.choice(SIZES))
        dt = DTYPES[int(rng.integers(0, len(DTYPES)))]
        c = {"kind": kind, "size": size, "dt": dt}
        if kind == 0:
            c["op"] = OPS[int(rng.integers(0, 4 if np.dtype(dt).kind != "f" else 3))]
        elif kind == 1:
            c["root"] = int(rng.integers(0, world))
        else:
            c["sizes"] = [int(rng.integers(0, max(2, size // world + 2))) for _ in range(world)]
            c["start"] = int(rng.integers(0, max(sum(c["sizes"]), 1)))
        cases.append(c)
    return cases


def data_of(case, r, size, dt):
    g = np.random.default_rng([seed, case, r])
    hi = 100 // world if np.dtype(dt).itemsize == 1 else 1000
    return g.integers(0, hi, size=size).astype(dt)


counts = {"allreduce": 0, "broadcast": 0, "allgather": 0}
version, state = rabit.load_checkpoint()
first = state["next"] if version > 0 else 0
for case, c in enumerate(draw_cases()):
    if case < first:
        continue
    kind, size, dt = c["kind"], c["size"], c["dt"]
    if kind == 0:
        op = c["op"]
        mine = data_of(case, rank, size, dt)
        got = rabit.allreduce(mine, op)
        allv = np.stack([data_of(case, r, size, dt) for r in range(world)]) if size else None
        if size == 0:
            want = mine
        elif op == rabit.MAX:
            want = allv.max(axis=0)
        elif op == rabit.MIN:
            want = allv.min(axis=0)
        elif op == rabit.SUM:
            want = allv.sum(axis=0, dtype=dt)
        else:
            want = np.bitwise_or.reduce(allv, axis=0)
        assert got.dtype == want.dtype and np.array_equal(got, want), (case, "allreduce", size,
                                                                       dt, op)
        counts["allreduce"] += 1
    elif kind == 1:
        root = c["root"]
        src = data_of(case, root, size, dt)
        got = rabit.broadcast(src if rank == root else None, root)
        assert isinstance(got, np.ndarray) and np.array_equal(got, src), (case, "broadcast", size,
                                                                          root)
        counts["broadcast"] += 1
    else:
        sizes, start = c["sizes"], c["start"]
        total = sum(sizes)
        full = data_of(case, world, total, dt)  # the gathered buffer everyone must end with
        buf = np.zeros(total, dtype=dt)
        begin = (start + sum(sizes[:rank])) % max(total, 1)
        for i in range(sizes[rank]):  # this rank's slice, wrapping around the end
            buf[(begin + i) % total] = full[(begin + i) % total]
        if total > 0:
            core._LIB.RabitAllgather(buf.ctypes.data_as(ctypes.c_void_p), total, begin,
                                     sizes[rank], sizes[(rank - 1) % world],
                                     core.DTYPE_ENUM[buf.dtype])
        assert np.array_equal(buf, full), (case, "allgather", sizes, start)
        counts["allgather"] += 1
    if case % 10 == 9:
        rabit.checkpoint({"next": case + 1})  # bounds the result log; restarts resume here
rabit.finalize()
print("[%d] FUZZ OK %s" % (rank, counts), flush=True)
