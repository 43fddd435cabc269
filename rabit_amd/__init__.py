"""xrabit — MI355X-native Reliable Allreduce and Broadcast Interface.

    import rabit_amd as rabit
    rabit.init()                       # or launched by rabit_amd.launcher / torchrun
    a = rabit.allreduce(np.ones(3), rabit.SUM)
    rabit.finalize()

See core.py for the API, tracker.py / launcher.py for job launch.
"""
from .core import (BITOR, DTYPE_ENUM, DTYPE_ENUM__, MAX, MIN, PREP_ABS, PREP_COPY,  # noqa: F401
                   PREP_SCALE, PREP_SQUARE, SUM, allgather, allgather_slice, allreduce,
                   allreduce_prepared, broadcast, broadcast_tensor, checkpoint, engine_name,
                   finalize, get_device,
                   get_processor_name, get_rank, get_ring_prev_rank, get_world_size, init,
                   is_distributed, last_error, lazy_checkpoint, lib, load_checkpoint,
                   set_error_mode, stats, tracker_print, version_number, dump_trace,
                   checkpoint_tensors, load_checkpoint_tensors, symmetric_empty,
                   set_device_transport, set_phase_timing, allreduce_graphable, TRANSPORT_AUTO,
                   TRANSPORT_DIRECT, TRANSPORT_RCCL, link_probe, probe_allreduce,
                   PROBE_BASE, PROBE_DUAL_STORE, PROBE_NO_WAIT, set_zero_copy)

__version__ = "0.1.0"
