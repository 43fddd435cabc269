"""Every device transport API path on a single GPU: world-1 device ops are routed through the
transports (rabit_device_world1_transport=1) instead of the local short-cut, so a one-rank RCCL
communicator runs ncclAllReduce / ncclBroadcast / ncclAllGather / ncclAllToAll (BitOR) / grouped
broadcasts (variable wrapping allgather), and a one-peer direct group runs its barrier, reduce
and gather kernels.  At world 1 every result equals the input.  argv[1]: rccl | direct | auto."""
import ctypes
import sys

import torch

import rabit_amd as rabit

algo = sys.argv[1]
rabit.init(sys.argv[2:], lib="standard", rabit_device=0, rabit_world1_fastpath=0,
           rabit_device_world1_transport=1, rabit_device_algo=algo)
assert rabit.get_world_size() == 1
dev = torch.device("cuda", 0)
checked = 0
for dt in (torch.int8, torch.uint8, torch.int32, torch.int64, torch.float32, torch.float64,
           torch.float16, torch.bfloat16):
    ops = [rabit.MAX, rabit.MIN, rabit.SUM] + ([rabit.BITOR] if not dt.is_floating_point else [])
    for op in ops:
        for n in (1, 1000, 65536 + 3, (3 << 20) // torch.tensor([], dtype=dt).element_size() + 5):
            v = (torch.arange(n, dtype=torch.int64) % 97 - 40).to(dt)
            if not dt.is_signed and not dt.is_floating_point:
                v = torch.arange(n, dtype=torch.int64).remainder(200).to(dt)
            t = v.to(dev)
            rabit.allreduce(t, op)
            assert torch.equal(t.cpu(), v), (algo, dt, op, n)
            checked += 1
# fused prepare: one rank, dst = src^2
src = torch.arange(1 << 20, device=dev, dtype=torch.float32).remainder_(17)
dst = torch.empty_like(src)
rabit.allreduce_prepared(dst, src, rabit.SUM, rabit.PREP_SQUARE)
assert torch.equal(dst, src * src), "prepared"
# broadcast (odd and large sizes)
for nbytes in (5, (5 << 20) + 3):
    b = torch.arange(nbytes, device=dev, dtype=torch.int64).remainder_(251).to(torch.uint8)
    want = b.clone()
    rabit.broadcast_tensor(b, 0)
    assert torch.equal(b, want), ("broadcast", nbytes)
# allgather: a uniform slice, then a wrapping one (begin != 0: the grouped path)
g = rabit.allgather(torch.arange(1000, device=dev, dtype=torch.float32))
assert torch.equal(g.cpu(), torch.arange(1000).float())
buf = torch.arange(777, device=dev, dtype=torch.int64).remainder_(200).to(torch.uint8)
want = buf.clone()
rabit.core._sync_stream_for(buf)
rabit.lib().RabitAllgather(ctypes.c_void_p(buf.data_ptr()), 777, 100, 777, 777, 1)
torch.cuda.synchronize()
assert torch.equal(buf, want), "allgatherv wrap"
st = rabit.stats()
want_rccl = algo in ("rccl", "auto")
assert st["device_rccl"] == (1 if want_rccl else 0), st
assert st["device_direct"] == (1 if algo in ("direct", "auto") else 0), st
tuning = st.get("rccl_tuning", {})
if any(a.startswith("rabit_rccl_tune=1") for a in sys.argv[2:]) and want_rccl:
    # the channel tuning timed RCCL's own choice and every candidate, kept one communicator
    assert set(tuning.get("us", {})) == {"rccl", "4", "16"}, tuning
    assert all(t > 0 for t in tuning["us"].values()), tuning
    assert tuning["chosen"] in tuning["us"], tuning
rabit.checkpoint(None)
rabit.finalize()
print("TRANSPORT1 OK algo=%s cases=%d calib=%s tuning=%s" % (algo, checked, st.get("calib_us"),
                                                             tuning), flush=True)
