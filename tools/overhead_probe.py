"""Host overhead of one world-1 device allreduce through the robust engine: the Python wrapper
vs a raw ctypes call vs the GPU work alone (async, so the loop rate is the host rate when the
host is slower than the GPU)."""
import ctypes
import json
import sys
import time

import torch

import rabit_amd as rabit

if "--torchrun" in sys.argv:  # as bench.py starts it: tracker in-process, world 1
    from rabit_amd.torchrun import init_from_env
    init_from_env(lib="standard", rabit_world1_fastpath=0, rabit_device=0)
else:
    rabit.init([], lib="standard", rabit_world1_fastpath=0)
L = rabit.lib()
dev = torch.device("cuda", 0)
res = {}
for n in (256, 32 << 20):
    x = torch.ones(n, device=dev)
    N = 300 if n < (1 << 20) else 100
    rabit.checkpoint(None)  # clears the HBM result log
    for _ in range(20):
        rabit.allreduce(x, rabit.SUM)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(N):
        rabit.allreduce(x, rabit.SUM)
    res["py_wrapper_issue_us_n%d" % n] = (time.perf_counter() - t0) / N * 1e6
    torch.cuda.synchronize()
    res["py_wrapper_us_n%d" % n] = (time.perf_counter() - t0) / N * 1e6
    ptr = ctypes.c_void_p(x.data_ptr())
    cb = L.PREPARE_FN()
    rabit.checkpoint(None)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(N):
        L.RabitAllreduce(ptr, n, 6, 2, cb, None)
    torch.cuda.synchronize()
    res["raw_ctypes_us_n%d" % n] = (time.perf_counter() - t0) / N * 1e6
    y = torch.empty_like(x)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(N):
        y.copy_(x)
    torch.cuda.synchronize()
    res["torch_copy_us_n%d" % n] = (time.perf_counter() - t0) / N * 1e6
    t0 = time.perf_counter()
    for _ in range(N):
        torch.cuda.current_stream(dev).cuda_stream
    res["py_current_stream_us"] = (time.perf_counter() - t0) / N * 1e6
print(json.dumps({k: round(v, 2) for k, v in res.items()}))
rabit.finalize()
