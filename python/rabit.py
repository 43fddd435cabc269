"""Drop-in module for code written against the reference's `python/rabit.py`: scripts that do
`sys.path.append('<rabit>/python'); import rabit` get xrabit's binding (rabit_amd.core) with
the same names: init(args, lib, lib_dll), finalize, get_rank, get_world_size, tracker_print,
get_processor_name, broadcast, allreduce, load_checkpoint, checkpoint, version_number and the
MAX/MIN/SUM/BITOR constants (reference python/rabit.py:83-364), plus xrabit's extensions."""
import os as _os
import sys as _sys

_ROOT = _os.path.dirname(_os.path.dirname(_os.path.abspath(__file__)))
if _ROOT not in _sys.path:
    _sys.path.insert(0, _ROOT)

from rabit_amd.core import *  # noqa: E402,F401,F403
from rabit_amd.core import (BITOR, DTYPE_ENUM__, MAX, MIN, SUM,  # noqa: E402,F401
                            allgather, allreduce, broadcast, checkpoint, finalize,
                            get_processor_name, get_rank, get_ring_prev_rank, get_world_size,
                            init, is_distributed, lazy_checkpoint, load_checkpoint, tracker_print,
                            version_number)
