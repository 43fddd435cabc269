"""Multi-rank HBM collectives through the direct (IPC peer-memory) transport.

All ranks share GPU 0 of the test box (RCCL refuses that, the direct transport does not), so
this drives the same code path as 8 ranks on 8 GPUs: stage -> flag barrier -> multi-source
reduce of peer segments -> barrier -> gather.  A 1 MiB stage buffer forces chunking.
Expected values are computed independently on the host with numpy."""
import ctypes
import os
import sys
import time

import numpy as np
import torch

import rabit_amd as rabit

lib = os.environ.get("XR_LIB", "standard")
rabit.init(sys.argv[1:], lib=lib, rabit_device=0, rabit_device_peer_buffer="1M",
           rabit_device_peer_timeout_sec=20)
rank, world = rabit.get_rank(), rabit.get_world_size()
dev = torch.device("cuda", 0)

TORCH = {
    np.int8: torch.int8, np.uint8: torch.uint8, np.int32: torch.int32, np.int64: torch.int64,
    np.float32: torch.float32, np.float64: torch.float64,
}


def values(r, n, dt, op):
    i = np.arange(n, dtype=np.int64)
    if op == rabit.BITOR:
        v = (1 << (r % 7)) | (i % 3)
    elif op == rabit.SUM:
        v = (i % 5) + r
    else:
        v = ((i * 7 + r * 13) % 29) - (10 if np.dtype(dt).kind != "u" else 0)
    return v.astype(dt)


def expected(n, dt, op):
    vs = [values(r, n, dt, op) for r in range(world)]
    if op == rabit.SUM:
        return np.sum(np.stack(vs).astype(np.float64), axis=0).astype(dt)
    if op == rabit.MAX:
        return np.max(np.stack(vs), axis=0)
    if op == rabit.MIN:
        return np.min(np.stack(vs), axis=0)
    out = vs[0]
    for v in vs[1:]:
        out = out | v
    return out


checked = 0
for dt in (np.int8, np.uint8, np.int32, np.int64, np.float32, np.float64):
    ops = [rabit.MAX, rabit.MIN, rabit.SUM]
    if np.dtype(dt).kind in "iu":
        ops.append(rabit.BITOR)
    for op in ops:
        for n in (1, 7, 1000, 65536 + 3, (3 << 20) // np.dtype(dt).itemsize + 5):
            t = torch.from_numpy(values(rank, n, dt, op)).to(dev)
            rabit.allreduce(t, op)
            got = t.cpu().numpy()
            exp = expected(n, dt, op)
            assert np.array_equal(got, exp), (dt, op, n, got[:8], exp[:8])
            checked += 1

# a buffer at an odd element offset on odd ranks only (a view): the transport's choices stay the
# same on every rank, only how this rank touches its own memory changes
for dt in (np.float32, np.int8, np.float64):
    for op in (rabit.SUM, rabit.MAX):
        n = (3 << 20) // np.dtype(dt).itemsize + 5
        vals = torch.from_numpy(values(rank, n, dt, op)).to(dev)
        if rank % 2 == 1:
            t = torch.empty(n + 1, dtype=vals.dtype, device=dev)[1:]
            t.copy_(vals)
        else:
            t = vals
        rabit.allreduce(t, op)
        assert np.array_equal(t.cpu().numpy(), expected(n, dt, op)), ("unaligned", dt, op)
        checked += 1

# fused lazy-prepare: dst = sum over ranks of src^2
n = (1 << 19) + 11
src = torch.arange(n, device=dev, dtype=torch.float32).remainder_(17).add_(rank)
dst = torch.empty_like(src)
rabit.allreduce_prepared(dst, src, rabit.SUM, rabit.PREP_SQUARE)
ref = sum((torch.arange(n, dtype=torch.float64).remainder(17) + r) ** 2 for r in range(world))
assert torch.equal(dst.cpu().double(), ref), "prepared allreduce"

# broadcast from every root, odd sizes and a chunked one
for nbytes in (5, 4096 + 1, (1 << 20) * 2 + 3):
    for root in range(world):
        if rank == root:
            b = torch.arange(nbytes, device=dev, dtype=torch.int64).remainder_(251).to(torch.uint8)
        else:
            b = torch.zeros(nbytes, device=dev, dtype=torch.uint8)
        rabit.broadcast_tensor(b, root)
        exp = torch.arange(nbytes, dtype=torch.int64).remainder(251).to(torch.uint8)
        assert torch.equal(b.cpu(), exp), ("broadcast", nbytes, root)

# pipelined broadcasts (several chunks each) back to back with allreduces in between, roots
# changing every op: the stage parity each op hands to the next must keep every buffer a slower
# peer still reads intact (bcast_plan.h)
for i in range(6):
    root = (i * 3 + 1) % world
    nbytes = (3 << 20) + 977 * i
    pat = (torch.arange(nbytes, dtype=torch.int64) * (i + 3)).remainder(253).to(torch.uint8)
    b = pat.to(dev) if rank == root else torch.zeros(nbytes, device=dev, dtype=torch.uint8)
    rabit.broadcast_tensor(b, root)
    assert torch.equal(b.cpu(), pat), ("pipelined broadcast", i, root)
    a = torch.full(((3 << 19) + i,), float(rank + i), device=dev)
    rabit.allreduce(a, rabit.SUM)
    assert torch.all(a == float(sum(r + i for r in range(world)))).item(), ("allreduce after bcast", i)

# allgather: equal slices through the Python API ...
g = rabit.allgather(torch.full((1000,), float(rank), device=dev))
assert torch.equal(g.cpu(), torch.arange(world).repeat_interleave(1000).float())
# ... and rabit's variable slices through the C API (uint8, slice r has 100 + 37 r bytes)
sizes = [100 + 37 * r for r in range(world)]
begin = [sum(sizes[:r]) for r in range(world)]
total = sum(sizes)
buf = torch.zeros(total, device=dev, dtype=torch.uint8)
buf[begin[rank]:begin[rank] + sizes[rank]] = rank + 1
rabit.core._sync_stream_for(buf)
rabit.lib().RabitAllgather(ctypes.c_void_p(buf.data_ptr()), total, begin[rank], sizes[rank],
                           sizes[(rank - 1) % world], 1)
exp = torch.cat([torch.full((sizes[r],), r + 1, dtype=torch.uint8) for r in range(world)])
assert torch.equal(buf.cpu(), exp), "allgatherv"

stats = rabit.stats()
assert stats["device_direct"] == 1 and stats["device_rccl"] == 0, stats
assert stats["oneshot_ops"] > 0, stats  # the small cases took the one-shot path
fused_oneshot = not any(a == "rabit_device_fused_oneshot=0" for a in sys.argv[1:])
assert (stats["fused_oneshots"] > 0) == fused_oneshot, stats  # ...in the form asked for
# every broadcast above went direct, the large ones in several pipeline chunks
assert stats["direct_bcast_ops"] >= 3 * world + 6, stats
assert stats["direct_bcast_chunks"] > stats["direct_bcast_ops"], stats
if "rabit_device_direct_mode=push" in sys.argv:
    assert stats["direct_push"] == 1 and stats["push_chunks"] > 0, stats
if "rabit_device_direct_mode=pipelined" in sys.argv:
    # the two-shot ops went through the pipelined push form, several rounds each
    assert stats["direct_pipeline"] == 1 and stats["direct_push"] == 1, stats
    assert stats["pipelined_ops"] > 0 and stats["pipelined_rounds"] > 3 * stats["pipelined_ops"], stats

# a rough number for the log: 64 MiB fp32 sum, all ranks' traffic on the one shared GPU
x = torch.ones(16 << 20, device=dev)
rabit.allreduce(x, rabit.SUM)
torch.cuda.synchronize()
t0 = time.time()
for _ in range(5):
    rabit.allreduce(x, rabit.SUM)
torch.cuda.synchronize()
dt_ms = (time.time() - t0) / 5 * 1e3
if rank == 0:
    print("[%d] 64MiB direct allreduce on a shared GPU, world %d: %.2f ms" % (rank, world, dt_ms))
rabit.finalize()
print("[%d] DEVMULTI OK (%d allreduce cases)" % (rank, checked), flush=True)
