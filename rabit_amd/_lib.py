"""Loader for the in-tree native libraries (rabit_amd/lib/librabit*.so).

The reference's binding picks a library by name (`python/rabit.py:47-74`); the same names are
used here.  The libraries are built in-tree by `make` (or `__graft_entry__.build()`); a
missing library is an error, never a silent pure-Python fallback.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.path.join(_HERE, "lib")

LIB_NAMES = {
    "standard": "librabit.so",
    "robust": "librabit.so",
    "base": "librabit_base.so",
    "mpi": "librabit_base.so",  # no MPI here: the non-fault-tolerant RCCL/TCP engine replaces it
    "mock": "librabit_mock.so",
    "empty": "librabit_empty.so",
}


def lib_path(lib: str = "standard") -> str:
    if lib not in LIB_NAMES:
        raise ValueError("unknown rabit library %r (choose from %s)" % (lib, sorted(LIB_NAMES)))
    return os.path.join(LIB_DIR, LIB_NAMES[lib])


def load(lib: str = "standard") -> ctypes.CDLL:
    path = lib_path(lib)
    if not os.path.exists(path):
        raise ImportError(
            "xrabit native library %s is missing; build it with `make -j8` in the repository "
            "root (or `python -c 'import __graft_entry__ as g; g.build()'`)" % path)
    dll = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)
    _declare(dll)
    return dll


def source_hash(root: str = None) -> str:
    """sha256 of every library source under csrc/ (.cc, .h, .hip) concatenated in byte order of
    their paths: the value the Makefile compiles into RabitBuildInfo"""
    import hashlib

    root = root or os.path.dirname(_HERE)
    paths = []
    for d, _, files in os.walk(os.path.join(root, "csrc")):
        for f in files:
            if f.endswith((".cc", ".h", ".hip")):
                paths.append(os.path.relpath(os.path.join(d, f), root))
    h = hashlib.sha256()
    for p in sorted(paths, key=lambda s: s.encode()):
        with open(os.path.join(root, p), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


def build_info(lib: str = "standard") -> dict:
    """what the library was built from (no init needed), plus whether it matches the sources
    in this tree (`fresh`)"""
    import json

    info = json.loads(load(lib).RabitBuildInfo().decode())
    info["library"] = os.path.relpath(lib_path(lib), os.path.dirname(_HERE))
    info["fresh"] = info.get("src_sha256") == source_hash()
    return info


def _declare(d: ctypes.CDLL) -> None:
    c_int, c_size_t = ctypes.c_int, ctypes.c_size_t
    c_void_p, c_char_p = ctypes.c_void_p, ctypes.c_char_p
    c_ulong, c_double = ctypes.c_ulong, ctypes.c_double
    prep_t = ctypes.CFUNCTYPE(None, c_void_p)
    sig = {
        "RabitInit": (ctypes.c_bool, [c_int, ctypes.POINTER(c_char_p)]),
        "RabitFinalize": (ctypes.c_bool, []),
        "RabitGetRingPrevRank": (c_int, []),
        "RabitGetRank": (c_int, []),
        "RabitBuildInfo": (c_char_p, []),
        "RabitGetWorldSize": (c_int, []),
        "RabitIsDistributed": (c_int, []),
        "RabitTrackerPrint": (None, [c_char_p]),
        "RabitGetProcessorName": (None, [c_char_p, ctypes.POINTER(c_ulong), c_ulong]),
        "RabitBroadcast": (None, [c_void_p, c_ulong, c_int]),
        "RabitAllgather": (None, [c_void_p, c_size_t, c_size_t, c_size_t, c_size_t, c_int]),
        "RabitAllreduce": (None, [c_void_p, c_size_t, c_int, c_int, prep_t, c_void_p]),
        "RabitLoadCheckPoint": (c_int, [ctypes.POINTER(ctypes.POINTER(ctypes.c_char)),
                                        ctypes.POINTER(c_ulong),
                                        ctypes.POINTER(ctypes.POINTER(ctypes.c_char)),
                                        ctypes.POINTER(c_ulong)]),
        "RabitCheckPoint": (None, [c_char_p, c_ulong, c_char_p, c_ulong]),
        "RabitLazyCheckPoint": (None, [c_char_p, c_ulong]),
        "RabitVersionNumber": (c_int, []),
        "RabitLinkTag": (c_int, []),
        "RabitEngineName": (c_char_p, []),
        "RabitSetStream": (None, [c_void_p]),
        "RabitGetDevice": (c_int, []),
        "RabitIsDevicePointer": (c_int, [c_void_p]),
        "RabitDevAllreducePrepared": (None, [c_void_p, c_void_p, c_size_t, c_int, c_int, c_int,
                                             c_double]),
        "RabitSetErrorMode": (None, [c_int]),
        "RabitDevCheckPoint": (None, [c_int, ctypes.POINTER(c_void_p), ctypes.POINTER(c_size_t),
                                      c_char_p, c_ulong]),
        "RabitDevLoadCheckPoint": (c_int, [c_int, ctypes.POINTER(c_void_p),
                                           ctypes.POINTER(c_size_t),
                                           ctypes.POINTER(ctypes.POINTER(ctypes.c_char)),
                                           ctypes.POINTER(c_ulong)]),
        "RabitDevCheckPointEx": (None, [c_int, ctypes.POINTER(c_void_p),
                                        ctypes.POINTER(c_size_t), c_char_p, c_ulong, c_int,
                                        ctypes.POINTER(c_void_p), ctypes.POINTER(c_size_t)]),
        "RabitDevLoadCheckPointEx": (c_int, [c_int, ctypes.POINTER(c_void_p),
                                             ctypes.POINTER(c_size_t),
                                             ctypes.POINTER(ctypes.POINTER(ctypes.c_char)),
                                             ctypes.POINTER(c_ulong), c_int,
                                             ctypes.POINTER(c_void_p), ctypes.POINTER(c_size_t)]),
        "RabitDevSetTransport": (c_int, [c_int, c_int]),
        "RabitDevSetFused": (c_int, [c_int]),
        "RabitDevGraphAllreduce": (c_int, [c_void_p, c_size_t, c_int, c_int, c_void_p]),
        "RabitDevSetPhaseTiming": (c_int, [c_int]),
        "RabitDevLinkProbe": (c_int, [c_size_t, ctypes.POINTER(c_double), c_int]),
        "RabitDevProbeAllreduce": (c_int, [c_void_p, c_size_t, c_int, c_int, c_int]),
        "RabitDevSetZeroCopy": (c_int, [c_size_t]),
        "RabitGetLastError": (c_char_p, []),
        "RabitGetStats": (c_char_p, []),
        "RabitTraceDump": (c_int, [c_char_p]),
        "RabitDevReduce": (c_int, [c_void_p, c_void_p, c_size_t, c_int, c_int, c_void_p]),
        "RabitDevReduceMulti": (c_int, [c_void_p, ctypes.POINTER(c_void_p), c_int, c_size_t,
                                        c_int, c_int, c_void_p]),
        "RabitDevPrepare": (c_int, [c_void_p, c_void_p, c_void_p, c_size_t, c_int, c_int,
                                    c_double, c_void_p]),
        "RabitDevChecksum": (c_int, [c_void_p, c_size_t, c_void_p, c_void_p]),
        "RabitDevFill": (c_int, [c_void_p, c_size_t, c_int, c_double, c_void_p]),
        "RabitDevCopy": (c_int, [c_void_p, c_void_p, c_size_t, c_void_p]),
        "RabitDevSymmetricAlloc": (c_void_p, [c_size_t]),
    }
    for name, (res, args) in sig.items():
        f = getattr(d, name)
        f.restype = res
        f.argtypes = args
    d.PREPARE_FN = prep_t
