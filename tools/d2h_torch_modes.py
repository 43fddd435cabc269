"""Which D2H copies run on a DMA engine inside a torch process (run one mode per process under
rocprofv3 --kernel-trace --memory-copy-trace):
  torch    pinned.copy_(dev, non_blocking=True)
  hip      hipMemcpyAsync through ctypes after torch initialised the device
  hipnt    hipMemcpyAsync through ctypes in a process that never imported torch
  torchlib hipMemcpyAsync through torch's bundled libamdhip64, torch never imported
  envdiff  print the C-level environment torch.cuda initialisation adds"""
import ctypes
import sys

mode = sys.argv[1]
nbytes = 64 << 20
if mode == "torch":
    import torch
    src = torch.ones(nbytes // 4, device="cuda")
    dst = torch.empty(nbytes // 4, pin_memory=True)
    s = torch.cuda.Stream()
    for _ in range(4):
        with torch.cuda.stream(s):
            dst.copy_(src, non_blocking=True)
        s.synchronize()
    print("torch", float(dst[0]))
    del src, dst
    torch.cuda.synchronize()
    raise SystemExit(0)
if mode == "envdiff":
    libc = ctypes.CDLL(None)

    def cenv():
        environ = ctypes.POINTER(ctypes.c_char_p).in_dll(libc, "environ")
        out, i = {}, 0
        while environ[i]:
            k, _, v = environ[i].decode(errors="replace").partition("=")
            out[k] = v
            i += 1
        return out

    before = cenv()
    import torch
    torch.cuda.init()
    torch.ones(1, device="cuda")
    after = cenv()
    print("envdiff", {k: v for k, v in after.items() if before.get(k) != v})
    raise SystemExit(0)
if mode == "hip":
    import torch
    torch.cuda.init()
    torch.ones(1, device="cuda")
libname = "libamdhip64.so"
if mode == "torchlib":
    import importlib.util
    import os
    spec = importlib.util.find_spec("torch")
    libname = os.path.join(os.path.dirname(spec.origin), "lib", "libamdhip64.so")
hip = ctypes.CDLL(libname)
dev = ctypes.c_void_p()
host = ctypes.c_void_p()
stream = ctypes.c_void_p()
assert hip.hipSetDevice(0) == 0
assert hip.hipMalloc(ctypes.byref(dev), ctypes.c_size_t(nbytes)) == 0
assert hip.hipHostMalloc(ctypes.byref(host), ctypes.c_size_t(nbytes), 0) == 0
assert hip.hipStreamCreateWithFlags(ctypes.byref(stream), 1) == 0
for _ in range(4):
    assert hip.hipMemcpyAsync(host, dev, ctypes.c_size_t(nbytes), 2, stream) == 0
    assert hip.hipStreamSynchronize(stream) == 0
assert hip.hipStreamDestroy(stream) == 0
assert hip.hipHostFree(host) == 0
assert hip.hipFree(dev) == 0
print(mode, "ok")
