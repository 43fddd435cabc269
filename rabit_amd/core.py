"""Python API of xrabit.

Drop-in for the reference binding (`python/rabit.py:83-364`): init, finalize, get_rank,
get_world_size, tracker_print, get_processor_name, broadcast (pickled objects), allreduce
(numpy), load_checkpoint, checkpoint, version_number, with the MAX/MIN/SUM/BITOR constants.

MI355X extensions: `allreduce` also takes torch tensors; HBM (CUDA/HIP) tensors are reduced
in place over RCCL/xGMI and the CDNA4 kernels, ordered on torch's current stream.  Plus
`allgather`, `broadcast_tensor`, `allreduce_prepared` (fused lazy prepare), `lazy_checkpoint`,
`stats`, `engine_name`, `get_device`.
"""
from __future__ import annotations

import ctypes
import threading
import json
import pickle
import sys
from typing import Any, Callable, Optional, Sequence

import numpy as np

from . import _lib

MAX = 0
MIN = 1
SUM = 2
BITOR = 3

# prepare ops of allreduce_prepared (csrc/src/device/kernels.h)
PREP_COPY = 0
PREP_SQUARE = 1
PREP_SCALE = 2
PREP_ABS = 3

_LIB: Optional[ctypes.CDLL] = None
_LIB_NAME: Optional[str] = None

# numpy dtype -> rabit dtype enum (engine.h mpi::DataType)
DTYPE_ENUM = {
    np.dtype("int8"): 0,
    np.dtype("uint8"): 1,
    np.dtype("int32"): 2,
    np.dtype("uint32"): 3,
    np.dtype("int64"): 4,
    np.dtype("uint64"): 5,
    np.dtype("float32"): 6,
    np.dtype("float64"): 7,
    np.dtype("float16"): 10,  # extension: IEEE half (mpi::kHalf)
}
DTYPE_ENUM__ = DTYPE_ENUM  # reference spelling


def _torch_dtype_enum(t) -> int:
    import torch

    table = {torch.int8: 0, torch.uint8: 1, torch.int32: 2, torch.int64: 4, torch.float32: 6,
             torch.float64: 7, torch.float16: 10, torch.bfloat16: 11}
    for name, code in (("uint32", 3), ("uint64", 5)):
        if hasattr(torch, name):
            table[getattr(torch, name)] = code
    if t.dtype not in table:
        raise TypeError("dtype %s is not supported by rabit allreduce" % t.dtype)
    return table[t.dtype]


def _check_init():
    if _LIB is None:
        raise RuntimeError("rabit_amd.init() must be called first")


def _loadlib(lib: str = "standard", lib_dll=None):
    global _LIB, _LIB_NAME
    if lib_dll is not None:
        _lib._declare(lib_dll)
        _LIB, _LIB_NAME = lib_dll, "custom"
        return
    if _LIB is not None and _LIB_NAME == lib:
        return
    _LIB = _lib.load(lib)
    _LIB_NAME = lib


def _unloadlib():
    global _LIB, _LIB_NAME
    _LIB, _LIB_NAME = None, None


def init(args: Optional[Sequence] = None, lib: str = "standard", lib_dll=None, **params):
    """Initialise the engine.  `args` are "name=value" strings (e.g. sys.argv); keyword
    params are appended the same way (init(rabit_debug=1))."""
    if args is None:
        args = []
    args = [a if isinstance(a, bytes) else str(a).encode() for a in args]
    args += [("%s=%s" % (k, v)).encode() for k, v in params.items()]
    _loadlib(lib, lib_dll)
    _GENERATION[0] += 1
    arr = (ctypes.c_char_p * len(args))(*args)
    if not _LIB.RabitInit(len(args), arr):
        raise RuntimeError("rabit init failed: %s" % last_error())


def finalize():
    """Finalize the engine; call after all jobs finished."""
    if _LIB is None:
        return
    _LIB.RabitFinalize()
    _GENERATION[0] += 1
    _unloadlib()


def get_rank() -> int:
    _check_init()
    return _LIB.RabitGetRank()


def get_world_size() -> int:
    _check_init()
    return _LIB.RabitGetWorldSize()


def is_distributed() -> bool:
    _check_init()
    return bool(_LIB.RabitIsDistributed())


def get_ring_prev_rank() -> int:
    _check_init()
    return _LIB.RabitGetRingPrevRank()


def tracker_print(msg: Any):
    """Print a message on the tracker (fixes the reference's c_char_p.encode bug)."""
    _check_init()
    if not isinstance(msg, str):
        msg = str(msg)
    _LIB.RabitTrackerPrint(msg.encode("utf-8"))


def get_processor_name() -> bytes:
    _check_init()
    mxlen = 256
    length = ctypes.c_ulong()
    buf = ctypes.create_string_buffer(mxlen)
    _LIB.RabitGetProcessorName(buf, ctypes.byref(length), mxlen)
    return buf.value


def broadcast(data: Any, root: int) -> Any:
    """Broadcast a picklable object from root; non-roots may pass None."""
    _check_init()
    rank = get_rank()
    length = ctypes.c_ulong()
    payload = None
    if root == rank:
        assert data is not None, "need to pass in data when broadcasting"
        payload = pickle.dumps(data, protocol=pickle.HIGHEST_PROTOCOL)
        length.value = len(payload)
    _LIB.RabitBroadcast(ctypes.byref(length), ctypes.sizeof(ctypes.c_ulong), root)
    if root != rank:
        dptr = (ctypes.c_char * length.value)()
        _LIB.RabitBroadcast(ctypes.cast(dptr, ctypes.c_void_p), length.value, root)
        data = pickle.loads(dptr.raw)
    else:
        buf = ctypes.create_string_buffer(payload, len(payload))
        _LIB.RabitBroadcast(ctypes.cast(buf, ctypes.c_void_p), length.value, root)
    return data


def _is_torch(x) -> bool:
    mod = type(x).__module__
    return mod.startswith("torch") and "torch" in sys.modules and \
        isinstance(x, sys.modules["torch"].Tensor)


# the stream last passed to the engine, per thread (an engine belongs to one thread) and per
# init generation (a new engine starts on the default stream)
_STREAM_CACHE = threading.local()
_GENERATION = [0]


def _current_raw_stream(device):
    """torch's current HIP stream on `device` as an integer handle (the raw accessor costs
    ~0.2 us against ~2 us for torch.cuda.current_stream(...).cuda_stream)"""
    import torch

    raw = getattr(torch._C, "_cuda_getCurrentRawStream", None)
    if raw is not None:
        return raw(device.index if device.index is not None else torch.cuda.current_device())
    return torch.cuda.current_stream(device).cuda_stream


def _sync_stream_for(t):
    """Order device collectives after torch's current stream on t's device (the engine is told
    only when the stream changed since the last call)."""
    if t.is_cuda:
        s = (_GENERATION[0], _current_raw_stream(t.device))
        if getattr(_STREAM_CACHE, "last", None) != s:
            _LIB.RabitSetStream(ctypes.c_void_p(s[1]))
            _STREAM_CACHE.last = s


def allreduce(data, op: int, prepare_fun: Optional[Callable] = None):
    """Allreduce.  numpy arrays: returns the reduced array (a flattened copy, as the
    reference).  torch tensors: reduced in place (must be contiguous) and returned; HBM
    tensors take the RCCL/HIP path.  prepare_fun(data) runs first unless the result is
    recovered from peers after a failure."""
    _check_init()
    if _is_torch(data):
        if not data.is_contiguous():
            raise ValueError("allreduce needs a contiguous tensor")
        if op == BITOR and data.is_floating_point():
            raise TypeError("BITOR is not defined for floating point data")
        enum = _torch_dtype_enum(data)
        if data.is_cuda:
            _sync_stream_for(data)
        cb = _make_prepare(prepare_fun, data)
        _LIB.RabitAllreduce(ctypes.c_void_p(data.data_ptr()), data.numel(), enum, op, cb, None)
        return data
    if not isinstance(data, np.ndarray):
        raise TypeError("allreduce only takes numpy.ndarray or torch.Tensor")
    buf = data.ravel()
    if buf.base is data.base:
        buf = buf.copy()
    if buf.dtype not in DTYPE_ENUM:
        raise TypeError("data type %s not supported" % str(buf.dtype))
    if op == BITOR and buf.dtype.kind == "f":
        raise TypeError("BITOR is not defined for floating point data")
    cb = _make_prepare(prepare_fun, data)
    _LIB.RabitAllreduce(buf.ctypes.data_as(ctypes.c_void_p), buf.size, DTYPE_ENUM[buf.dtype], op,
                        cb, None)
    return buf


_NO_PREPARE = {}


def _make_prepare(prepare_fun, data):
    if prepare_fun is None:
        cb = _NO_PREPARE.get(id(_LIB))
        if cb is None:
            cb = _NO_PREPARE[id(_LIB)] = _LIB.PREPARE_FN()
        return cb

    def pfunc(_arg):
        prepare_fun(data)

    cb = _LIB.PREPARE_FN(pfunc)
    _make_prepare.keep = cb  # keep alive for the duration of the call
    return cb


def allreduce_prepared(dst, src, op: int, prep: int = PREP_SQUARE, alpha: float = 1.0):
    """Fused lazy-prepare allreduce of HBM tensors: dst = prep(src) (gfx950 kernel), then
    allreduce(dst).  The prepare kernel is skipped when the result is recovered."""
    _check_init()
    assert dst.is_cuda and src.is_cuda and dst.numel() == src.numel() and dst.dtype == src.dtype
    _sync_stream_for(dst)
    _LIB.RabitDevAllreducePrepared(ctypes.c_void_p(dst.data_ptr()), ctypes.c_void_p(src.data_ptr()),
                                   dst.numel(), _torch_dtype_enum(dst), op, prep, float(alpha))
    return dst


def broadcast_tensor(t, root: int):
    """In-place broadcast of a contiguous numpy array or torch tensor (host or HBM)."""
    _check_init()
    if _is_torch(t):
        if t.is_cuda:
            _sync_stream_for(t)
        _LIB.RabitBroadcast(ctypes.c_void_p(t.data_ptr()), t.numel() * t.element_size(), root)
        return t
    assert t.flags["C_CONTIGUOUS"]
    _LIB.RabitBroadcast(t.ctypes.data_as(ctypes.c_void_p), t.nbytes, root)
    return t


def allgather(data):
    """Gather equal-size slices from every rank: returns an array of world_size * len(data)
    (torch tensors stay on their device)."""
    _check_init()
    n, r = get_world_size(), get_rank()
    if _is_torch(data):
        import torch

        flat = data.contiguous().view(-1)
        out = torch.empty(n * flat.numel(), dtype=flat.dtype, device=flat.device)
        out[r * flat.numel():(r + 1) * flat.numel()] = flat
        if out.is_cuda:
            _sync_stream_for(out)
        _LIB.RabitAllgather(ctypes.c_void_p(out.data_ptr()), out.numel(), r * flat.numel(),
                            flat.numel(), flat.numel(), _torch_dtype_enum(out))
        return out
    flat = np.ascontiguousarray(data).ravel()
    out = np.empty(n * flat.size, dtype=flat.dtype)
    out[r * flat.size:(r + 1) * flat.size] = flat
    _LIB.RabitAllgather(out.ctypes.data_as(ctypes.c_void_p), out.size, r * flat.size, flat.size,
                        flat.size, DTYPE_ENUM[out.dtype])
    return out


def allgather_slice(data, begin: int, size: int, size_prev_slice: int = 0):
    """rabit's general Allgather, in place: this rank owns data[begin : begin + size] (element
    indices, wrapping modulo len(data)); afterwards data holds every rank's slice.  The slices
    of all ranks partition data, ring-ordered: the next rank's slice starts where this one ends
    (reference `include/rabit/rabit.h` Allgather).  A contiguous torch tensor (HBM or host) or
    numpy array; returned.  size_prev_slice: the previous rank's slice size (the host ring uses
    it; the device transports do not need it)."""
    _check_init()
    if _is_torch(data):
        if not data.is_contiguous():
            raise ValueError("allgather_slice needs a contiguous tensor")
        if data.is_cuda:
            _sync_stream_for(data)
        _LIB.RabitAllgather(ctypes.c_void_p(data.data_ptr()), data.numel(), int(begin),
                            int(size), int(size_prev_slice), _torch_dtype_enum(data))
        return data
    if not (isinstance(data, np.ndarray) and data.flags.c_contiguous):
        raise TypeError("allgather_slice takes a contiguous numpy array or torch tensor")
    _LIB.RabitAllgather(data.ctypes.data_as(ctypes.c_void_p), data.size, int(begin), int(size),
                        int(size_prev_slice), DTYPE_ENUM[data.dtype])
    return data


def _load_model(ptr, length):
    data = (ctypes.c_char * length).from_address(ctypes.addressof(ptr.contents))
    return pickle.loads(data.raw)


def load_checkpoint(with_local: bool = False):
    """Load the latest checkpoint: (version, global[, local]); version 0 means none."""
    _check_init()
    gptr = ctypes.POINTER(ctypes.c_char)()
    glen = ctypes.c_ulong()
    if with_local:
        lptr = ctypes.POINTER(ctypes.c_char)()
        llen = ctypes.c_ulong()
        version = _LIB.RabitLoadCheckPoint(ctypes.byref(gptr), ctypes.byref(glen),
                                           ctypes.byref(lptr), ctypes.byref(llen))
        if version == 0:
            return (version, None, None)
        return (version, _load_model(gptr, glen.value), _load_model(lptr, llen.value))
    version = _LIB.RabitLoadCheckPoint(ctypes.byref(gptr), ctypes.byref(glen), None, None)
    if version == 0:
        return (version, None)
    return (version, _load_model(gptr, glen.value))


def checkpoint(global_model: Any, local_model: Any = None):
    """Checkpoint (pickled) models; the version number increases by one."""
    _check_init()
    sglobal = pickle.dumps(global_model)
    if local_model is None:
        _LIB.RabitCheckPoint(sglobal, len(sglobal), None, 0)
    else:
        slocal = pickle.dumps(local_model)
        _LIB.RabitCheckPoint(sglobal, len(sglobal), slocal, len(slocal))


_lazy_keep = None


def lazy_checkpoint(global_model: Any):
    """Lazy checkpoint: the pickled bytes are kept and only sent if a peer needs them."""
    global _lazy_keep
    _check_init()
    _lazy_keep = pickle.dumps(global_model)
    _LIB.RabitLazyCheckPoint(_lazy_keep, len(_lazy_keep))


def _tensor_list(tensors):
    if tensors is None:
        tensors = []
    items = list(tensors.values()) if isinstance(tensors, dict) else list(tensors)
    for t in items:
        if not (_is_torch(t) and t.is_cuda and t.is_contiguous()):
            raise TypeError("device checkpoints take contiguous HBM (cuda) tensors")
    n = len(items)
    ptrs = (ctypes.c_void_p * max(n, 1))(*[t.data_ptr() for t in items])
    sizes = (ctypes.c_size_t * max(n, 1))(*[t.numel() * t.element_size() for t in items])
    return items, n, ptrs, sizes


def checkpoint_tensors(tensors, meta: Any = None, local=None):
    """Checkpoint HBM tensors (dict or list) plus a picklable `meta`: HBM snapshot with the
    gfx950 copy kernel and an asynchronous pinned-host mirror on a side stream; the bytes are
    only serialised if a recovering peer asks for them.  `local`: this rank's own tensors
    (its local model): kept in HBM together with the local models of its rabit_local_replica
    ring predecessors and replicated to its successors over xGMI, never through host memory.
    Version number += 1."""
    _check_init()
    items, n, ptrs, sizes = _tensor_list(tensors)
    litems, nl, lptrs, lsizes = _tensor_list(local)
    if items or litems:
        _sync_stream_for((items or litems)[0])
    m = pickle.dumps(meta)
    if local is None:
        _LIB.RabitDevCheckPoint(n, ptrs, sizes, m, len(m))
    else:
        _LIB.RabitDevCheckPointEx(n, ptrs, sizes, m, len(m), nl, lptrs, lsizes)


def load_checkpoint_tensors(tensors, local=None):
    """Fill HBM tensors (same order/shapes as checkpointed) from the latest device
    checkpoint, and this rank's `local` tensors from the replicated local checkpoint;
    returns (version, meta), version 0 = nothing checkpointed (tensors untouched)."""
    _check_init()
    items, n, ptrs, sizes = _tensor_list(tensors)
    litems, nl, lptrs, lsizes = _tensor_list(local)
    if items or litems:
        _sync_stream_for((items or litems)[0])
    mptr = ctypes.POINTER(ctypes.c_char)()
    mlen = ctypes.c_ulong()
    if local is None:
        version = _LIB.RabitDevLoadCheckPoint(n, ptrs, sizes, ctypes.byref(mptr),
                                              ctypes.byref(mlen))
    else:
        version = _LIB.RabitDevLoadCheckPointEx(n, ptrs, sizes, ctypes.byref(mptr),
                                                ctypes.byref(mlen), nl, lptrs, lsizes)
    if version <= 0:
        return (version, None)
    return (version, _load_model(mptr, mlen.value))


def version_number() -> int:
    _check_init()
    return _LIB.RabitVersionNumber()


# ----------------------------------------------------------------------------- extensions
def engine_name() -> str:
    _check_init()
    return _LIB.RabitEngineName().decode()


def get_device() -> int:
    _check_init()
    return _LIB.RabitGetDevice()


def stats() -> dict:
    _check_init()
    return json.loads(_LIB.RabitGetStats().decode())


def dump_trace(path: str) -> int:
    """Write the engine's span log (init with rabit_trace=1) as a Chrome trace JSON file;
    returns the number of spans."""
    _check_init()
    return _LIB.RabitTraceDump(path.encode())


TRANSPORT_AUTO = -1
TRANSPORT_RCCL = 0
TRANSPORT_DIRECT = 1


def set_device_transport(which: int = TRANSPORT_AUTO, direct_mode: Optional[str] = None,
                         fused: Optional[bool] = None) -> bool:
    """Route this rank's device collectives over one transport (benchmarks / diagnosis):
    TRANSPORT_AUTO (the calibrated choice), TRANSPORT_RCCL or TRANSPORT_DIRECT, pick the
    direct reduce-scatter variant ("pull" / "push" / "pipelined": push whose rounds also carry
    the gather of an older chunk, over the opposite link direction) and the form of the direct
    two-shot path (fused=True: one kernel per chunk with per-tile hand-offs; False: the 5-launch
    form).
    Every rank must make the same call between the same collectives.  False when that
    transport is not up on this rank."""
    _check_init()
    mode = {None: 0, "pull": 1, "push": 2, "pipelined": 3}[direct_mode]
    if _LIB.RabitDevSetTransport(int(which), mode) != 0:
        return False
    if fused is not None:
        return _LIB.RabitDevSetFused(1 if fused else 0) == 0
    return True


LINK_PROBE_KEYS = ("one_link_read_GBps", "one_link_write_GBps", "all_links_read_GBps",
                   "all_links_write_GBps", "all_links_both_ways_GBps")


def link_probe(nbytes: int = 64 << 20) -> Optional[dict]:
    """xGMI link bandwidth of this rank over the direct transport's IPC mappings (a collective
    outside the fault-tolerance log: every rank calls it between the same ops).  Copies of
    `nbytes` (at most one stage buffer), each right after a barrier: one link read / write (every
    rank to rank + k at once, mean over k), all links read / write (1/(n-1) of the bytes to or
    from each peer at once), all links both ways at once.  GB/s per direction of this rank; None
    without a direct transport (world 1, ranks on several hosts).  Raises RuntimeError if a peer
    failed during the probe (the next collective rebuilds the transport)."""
    _check_init()
    out = (ctypes.c_double * 5)()
    r = _LIB.RabitDevLinkProbe(int(nbytes), out, 5)
    if r == -2:
        return None
    if r != 0:
        raise RuntimeError("link probe failed: " + last_error())
    return {k: round(float(v), 2) for k, v in zip(LINK_PROBE_KEYS, out)}


def set_zero_copy(min_bytes: int) -> bool:
    """Ordinary HBM inputs of at least min_bytes are IPC-registered and read in place by the
    direct transport's peers instead of being staged (default 1 MiB; 0 turns it off).  Every
    rank must make the same call between the same collectives.  False without a device plane."""
    _check_init()
    return _LIB.RabitDevSetZeroCopy(int(min_bytes)) == 0


PROBE_BASE, PROBE_DUAL_STORE, PROBE_NO_WAIT = 0, 1, 2


def probe_allreduce(t, op: int, mode: int = PROBE_BASE):
    """The fault-tolerance tax, measured: the device allreduce the robust engine runs, on the
    same transports and routing, but outside its result log and sequence numbering (a
    collective every rank calls between the same ops, like link_probe; for benchmarks -- a
    failure raises RuntimeError and is not recovered).  mode PROBE_BASE: in place with the host
    wait, what the base engine runs; PROBE_DUAL_STORE: into a scratch slot and t, as the robust
    engine stores into its log and the user buffer; PROBE_NO_WAIT: in place, stream-ordered."""
    _check_init()
    if not (_is_torch(t) and t.is_cuda and t.is_contiguous()):
        raise TypeError("probe_allreduce takes a contiguous HBM (cuda) tensor")
    _sync_stream_for(t)
    r = _LIB.RabitDevProbeAllreduce(ctypes.c_void_p(t.data_ptr()), t.numel(),
                                    _torch_dtype_enum(t), int(op), int(mode))
    if r != 0:
        raise RuntimeError("probe_allreduce failed (%d): %s" % (r, last_error()))
    return t


def allreduce_graphable(t, op: int):
    """In-place allreduce of an HBM tensor on the current stream, with no host-side
    synchronisation: unlike allreduce(), it can be captured into a hipGraph with the rest of
    the step (torch.cuda.graph / rabit_amd.parallel.GraphedStep).  It runs over RCCL, or over
    the direct transport (classic form, barriers numbered on the device so every replay
    resynchronises) when the routing sends this size there or RCCL is not up.  Graph replays
    and other collectives must be ordered on the GPU (one stream, or joined streams).  Make one
    eager call before capturing (it brings the transports up).  Non-fault-tolerant engines only
    (init(lib="base")): the op has no sequence number, result log or replay.  Identity at world
    size 1 without a device transport."""
    import torch

    _check_init()
    if not (_is_torch(t) and t.is_cuda and t.is_contiguous()):
        raise TypeError("allreduce_graphable takes a contiguous HBM (cuda) tensor")
    stream = torch.cuda.current_stream(t.device).cuda_stream
    r = _LIB.RabitDevGraphAllreduce(t.data_ptr(), t.numel(), _torch_dtype_enum(t), int(op),
                                    stream)
    if r != 0:
        raise RuntimeError("allreduce_graphable: %s" % last_error())
    return t


def set_phase_timing(on: bool) -> bool:
    """Time the phases of the direct transport's classic two-shot allreduce (stage, barrier,
    reduce, barrier, gather) with hipEvents from now on, with fresh totals (on=True), or stop.
    Averages per op appear in stats()["direct_phase_us"].  False without a direct transport."""
    _check_init()
    return _LIB.RabitDevSetPhaseTiming(1 if on else 0) == 0


def last_error() -> str:
    if _LIB is None:
        return ""
    return _LIB.RabitGetLastError().decode()


def set_error_mode(raise_errors: bool):
    """raise_errors=False (default): a native error exits the process (the launcher restarts
    the worker).  True: errors are raised as RuntimeError instead (tests)."""
    _check_init()
    _LIB.RabitSetErrorMode(1 if raise_errors else 0)


class _DeviceArray:
    """__cuda_array_interface__ view of engine-owned HBM (torch.as_tensor wraps it zero-copy)."""

    def __init__(self, ptr: int, shape, typestr: str, owner):
        self.__cuda_array_interface__ = {"shape": tuple(shape), "typestr": typestr,
                                         "data": (ptr, False), "version": 2, "strides": None}
        self._owner = owner


def symmetric_empty(shape, dtype=None):
    """A torch tensor in the engine's symmetric heap (init with rabit_device_symmetric_heap=...).

    Peers map this memory through IPC, so allreducing a tensor allocated here skips the staging
    copy of the direct transport.  The memory belongs to the engine (valid until finalize())."""
    import torch

    _check_init()
    dtype = dtype or torch.float32
    if isinstance(shape, int):
        shape = (shape,)
    numel = 1
    for d in shape:
        numel *= int(d)
    esize = torch.empty((), dtype=dtype).element_size()
    ptr = _LIB.RabitDevSymmetricAlloc(max(1, numel * esize))
    if not ptr:
        raise MemoryError("symmetric heap unavailable or full (rabit_device_symmetric_heap)")
    typestr = {torch.float32: "<f4", torch.float64: "<f8", torch.int32: "<i4",
               torch.int64: "<i8", torch.uint8: "|u1", torch.int8: "|i1",
               torch.float16: "<f2", torch.bfloat16: "<i2"}[dtype]
    dev = torch.device("cuda", get_device())
    with torch.cuda.device(dev):
        t = torch.as_tensor(_DeviceArray(ptr, shape, typestr, None), device=dev)
    if dtype == torch.bfloat16:  # no array-interface code for bf16: same bits as int16
        t = t.view(torch.bfloat16)
    assert t.data_ptr() == ptr, "torch copied the symmetric buffer"
    return t


def lib():
    """The loaded ctypes library (for rabit_amd.ops)."""
    return _LIB
