"""Initialise rabit inside a `torch.distributed.run` (torchrun) job.

torchrun gives every process RANK / WORLD_SIZE / LOCAL_RANK / MASTER_ADDR / MASTER_PORT but
no rabit tracker.  Rank 0 hosts the tracker in a background thread on a free port from
MASTER_PORT + offset on and publishes it in torchrun's agent store (outside torchrun: exactly
MASTER_PORT + offset);
every rank joins with its torchrun RANK as task id, so the tracker's batch assignment (ordered
by host, then numeric task id) gives rabit rank == torchrun RANK on a single node, and the
device plane picks the GPU from LOCAL_RANK (one process per GPU, RCCL over xGMI).
"""
from __future__ import annotations

import os
from typing import Optional

from . import core as rabit
from .tracker import RabitTracker

TRACKER_PORT_OFFSET = 17


class TorchrunContext:
    def __init__(self, rank: int, world: int, local_rank: int, tracker: Optional[RabitTracker]):
        self.rank, self.world, self.local_rank, self.tracker = rank, world, local_rank, tracker

    def finalize(self, timeout: float = 60.0):
        rabit.finalize()
        if self.tracker is not None:
            self.tracker.join(timeout)


def _node_has_gpus() -> bool:
    try:
        import torch
        return torch.cuda.device_count() > 0  # counts devices without initialising HIP
    except Exception:  # noqa: BLE001
        return False


def _agent_store(addr: str, port: int):
    """a client of the TCPStore torchrun's agent serves at MASTER_ADDR:MASTER_PORT (the store
    torch.distributed's env:// rendezvous uses under torchrun), or None outside torchrun"""
    if os.environ.get("TORCHELASTIC_USE_AGENT_STORE", "").lower() != "true":
        return None
    try:
        from datetime import timedelta

        from torch.distributed import TCPStore
        return TCPStore(addr, port, is_master=False, timeout=timedelta(seconds=300))
    except Exception:  # noqa: BLE001 - fall back to the fixed port offset
        return None


def init_from_env(lib: str = "standard", port_offset: int = TRACKER_PORT_OFFSET,
                  **params) -> TorchrunContext:
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    addr = os.environ.get("MASTER_ADDR", "127.0.0.1")
    master_port = int(os.environ.get("MASTER_PORT", "29500"))
    tracker = None
    if world == 1 and "MASTER_PORT" not in os.environ:
        # standalone single process: any free port
        tracker = RabitTracker(addr, 1, port=9091, port_end=9591, print_fn=lambda m: None)
        tracker.start(1)
        port = tracker.port
    else:
        store = _agent_store(addr, master_port)
        if store is not None:
            # torchrun's own store carries the tracker port: rank 0 binds any free port near
            # MASTER_PORT + offset and publishes it (keyed by the restart round)
            key = "xrabit/tracker_port/%s" % os.environ.get("TORCHELASTIC_RESTART_COUNT", "0")
            if rank == 0:
                start = master_port + port_offset
                tracker = RabitTracker(addr, world, port=start, port_end=start + 200,
                                       print_fn=lambda m: None)
                tracker.start(world)
                store.set(key, str(tracker.port))
            port = int(store.get(key).decode())
        else:
            port = master_port + port_offset
            if rank == 0:
                tracker = RabitTracker(addr, world, port=port, port_end=port + 1,
                                       print_fn=lambda m: None)
                tracker.start(world)
    args = dict(rabit_tracker_uri=addr, rabit_tracker_port=port, rabit_task_id=rank,
                rabit_world_size=world, DMLC_WORKER_CONNECT_RETRY=30)
    if "rabit_device" not in params:
        params["rabit_device"] = local_rank
    if "rabit_host_via_device" not in params and _node_has_gpus():
        # one process per GPU: every rank has a device plane, so large host-buffer allreduces
        # can uniformly take the HBM transports (staged over PCIe) instead of loopback TCP
        params["rabit_host_via_device"] = 1
    args.update(params)
    # extra engine parameters for every rank of a launched job: XRABIT_PARAMS="k=v,k=v"
    # (rehearsals and tuning runs; explicit keyword parameters win)
    for kv in filter(None, os.environ.get("XRABIT_PARAMS", "").split(",")):
        k, _, v = kv.partition("=")
        if k and k not in params:
            args[k.strip()] = v.strip()
    rabit.init(lib=lib, **args)
    assert rabit.get_world_size() == world, "rabit world size differs from torchrun's"
    return TorchrunContext(rank, world, local_rank, tracker)
