"""Direct access to the gfx950 kernels of the device data plane (csrc/src/device/kernels.hip).

These are the building blocks the engine uses for HBM buffers: element-wise reduce (K1-K4 of
SURVEY §2.11), multi-source reduce (local step of the all-to-all allreduce used for BitOR),
fused lazy prepare (K8) and a position-weighted checksum.  All functions take torch CUDA/HIP
tensors and enqueue on torch's current stream.  They raise if the native library is missing
(there is no silent eager fallback).
"""
from __future__ import annotations

import ctypes
from typing import Sequence

from .. import _lib

MAX, MIN, SUM, BITOR = 0, 1, 2, 3
PREP_COPY, PREP_SQUARE, PREP_SCALE, PREP_ABS = 0, 1, 2, 3

_DLL = None


def _dll():
    global _DLL
    if _DLL is None:
        _DLL = _lib.load("standard")
    return _DLL


def dtype_enum(t) -> int:
    import torch

    table = {torch.int8: 0, torch.uint8: 1, torch.int32: 2, torch.int64: 4, torch.float32: 6,
             torch.float64: 7, torch.float16: 10, torch.bfloat16: 11}
    for name, code in (("uint32", 3), ("uint64", 5)):
        if hasattr(torch, name):
            table[getattr(torch, name)] = code
    return table[t.dtype]


def _stream(t):
    import torch

    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def _check(rc: int, what: str):
    if rc != 0:
        raise RuntimeError("%s failed with hipError %d" % (what, rc))


def reduce_(dst, src, op: int):
    """dst = op(dst, src) in place."""
    assert dst.is_cuda and src.is_cuda and dst.numel() == src.numel() and dst.dtype == src.dtype
    _check(_dll().RabitDevReduce(ctypes.c_void_p(dst.data_ptr()), ctypes.c_void_p(src.data_ptr()),
                                 dst.numel(), dtype_enum(dst), op, _stream(dst)), "RabitDevReduce")
    return dst


def reduce_multi(dst, srcs: Sequence, op: int):
    """dst = op(srcs[0], ..., srcs[k-1]), k <= 8 (dst may be srcs[0])."""
    k = len(srcs)
    arr = (ctypes.c_void_p * k)(*[s.data_ptr() for s in srcs])
    _check(_dll().RabitDevReduceMulti(ctypes.c_void_p(dst.data_ptr()), arr, k, dst.numel(),
                                      dtype_enum(dst), op, _stream(dst)), "RabitDevReduceMulti")
    return dst


def prepare(dst, src, prep: int, alpha: float = 1.0, dst2=None):
    """dst (and dst2) = prep(src) in one pass."""
    _check(_dll().RabitDevPrepare(ctypes.c_void_p(dst.data_ptr()),
                                  ctypes.c_void_p(dst2.data_ptr() if dst2 is not None else 0),
                                  ctypes.c_void_p(src.data_ptr()), dst.numel(), dtype_enum(dst),
                                  prep, float(alpha), _stream(dst)), "RabitDevPrepare")
    return dst


def checksum(buf, out=None):
    """(sum of 32-bit words, sum of (i+1)*word) mod 2^64 over the tensor's bytes, as a 2-element
    int64 tensor; with `out` (zeroed int64[2] on the device) the sums are ADDED to it."""
    import torch

    if out is None:
        out = torch.zeros(2, dtype=torch.int64, device=buf.device)
    _check(_dll().RabitDevChecksum(ctypes.c_void_p(buf.data_ptr()),
                                   buf.numel() * buf.element_size(),
                                   ctypes.c_void_p(out.data_ptr()), _stream(buf)),
           "RabitDevChecksum")
    return out


def copy(dst, src):
    """dst <- src (bytes of src), gfx950 copy kernel."""
    nbytes = src.numel() * src.element_size()
    assert dst.numel() * dst.element_size() >= nbytes
    _check(_dll().RabitDevCopy(ctypes.c_void_p(dst.data_ptr()), ctypes.c_void_p(src.data_ptr()),
                               nbytes, _stream(dst)), "RabitDevCopy")
    return dst


def fill(dst, value: float):
    _check(_dll().RabitDevFill(ctypes.c_void_p(dst.data_ptr()), dst.numel(), dtype_enum(dst),
                               float(value), _stream(dst)), "RabitDevFill")
    return dst
