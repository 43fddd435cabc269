"""Registered zero copy of ordinary torch allocations over the direct transport (ranks share
GPU 0): peers read every rank's input in place once its allocation is IPC-registered
(csrc/src/device/peer_registry.h), including
  * the same buffer with new values every op (a reader must never see the previous op's bytes),
  * a sub-view at an offset, an unaligned view (staged) and a multi-chunk op,
  * the allocation freed (empty_cache: the segment goes back to the driver) and a new one made,
    likely at the same address, between ops,
  * more live allocations than registry slots, cycled (slots are evicted and remapped).
Every result is checked bit for bit against the closed form.  argv: mode=pull|push ..."""
import os
import sys

import torch

import rabit_amd as rabit

args = [a for a in sys.argv[1:]]
rabit.init(args, lib="standard", rabit_device=0, rabit_device_peer_buffer="8M",
           rabit_device_peer_timeout_sec=30)
rank, world = rabit.get_rank(), rabit.get_world_size()
dev = torch.device("cuda", 0)
ops = 0


def phase(msg):
    print("[%d] phase %s registry %s" % (rank, msg, rabit.stats()["zero_copy_registry"]), flush=True)


def check(x, tag, seed):
    """allreduce(SUM) of (base + seed + rank) into x, compare with the closed form"""
    global ops
    n = x.numel()
    base = torch.arange(n, device=dev, dtype=torch.float64).remainder(13)
    x.copy_((base + seed + rank).to(x.dtype))
    rabit.allreduce(x, rabit.SUM)
    want = (base + seed) * world + world * (world - 1) / 2
    assert torch.equal(x.double(), want), (tag, seed, n)
    ops += 1


# 1. one buffer reused with new values each op (3 chunks of the 8 MiB stage)
x = torch.empty(5 << 20, dtype=torch.float32, device=dev)
for it in range(8):
    check(x, "reuse", it)
phase("reuse done")
st = rabit.stats()
reg1 = st["zero_copy_registry"]
# 2. views into the same allocation: aligned offset (zero copy), unaligned (staged)
for it in range(4):
    check(x[4096:4096 + (2 << 20)], "view", 100 + it)
    check(x[3:3 + (2 << 20)], "unaligned", 200 + it)
phase("views done")
# 3. free the segment and allocate again (same size: often the same address, new buffer id)
del x
torch.cuda.synchronize()
torch.cuda.empty_cache()
y = torch.empty(5 << 20, dtype=torch.float32, device=dev)
for it in range(6):
    check(y, "realloc", 300 + it)
del y
torch.cuda.synchronize()
torch.cuda.empty_cache()
phase("realloc done")
# 4. 40 live allocations (> 32 registry slots) of 12 MiB, each its own segment, cycled twice
bufs = [torch.empty(3 << 20, dtype=torch.float32, device=dev) for _ in range(40)]
for rnd in range(2):
    for i, b in enumerate(bufs):
        check(b, "cycle", 1000 + 50 * rnd + i)
phase("cycle done")
# 5. other dtypes and MAX on a reused buffer
z = torch.empty(3 << 20, dtype=torch.int32, device=dev)
for it in range(4):
    base = torch.arange(z.numel(), device=dev, dtype=torch.int64).remainder(11)
    z.copy_((base * (rank + 1) + it).to(torch.int32))
    rabit.allreduce(z, rabit.MAX)
    assert torch.equal(z.long(), base * world + it), ("max", it)
    ops += 1
torch.cuda.synchronize()
st = rabit.stats()
reg = st["zero_copy_registry"]
zc_off = "rabit_device_zero_copy=0" in args
# torch's expandable segments are VMM allocations: the registry either maps them (the runtime
# exports them) or finds them unexportable and stages them; the results are exact either way
vmm = "expandable_segments:True" in os.environ.get("PYTORCH_HIP_ALLOC_CONF", "")
if world > 1 and zc_off:
    assert reg["zero_copy_chunks"] == 0 and reg["exports"] == 0, reg
if world > 1 and vmm:
    assert reg["opened"] and (reg["unexportable"] > 0 or reg["zero_copy_chunks"] > 0), reg
elif world > 1 and "rabit_device_direct_mode=push" not in args and not zc_off:
    assert reg["opened"], reg
    assert reg1["zero_copy_chunks"] > 0, reg1
    assert reg["zero_copy_chunks"] > 0 and reg["exports"] >= 3 and reg["imports"] >= 3, reg
rabit.finalize()
print("[%d] ZEROCOPY OK %d ops registry %s" % (rank, ops, reg), flush=True)
