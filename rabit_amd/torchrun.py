"""Initialise rabit inside a `torch.distributed.run` (torchrun) job.

torchrun gives every process RANK / WORLD_SIZE / LOCAL_RANK / MASTER_ADDR / MASTER_PORT but
no rabit tracker.  Rank 0 hosts the tracker in a background thread at MASTER_PORT + offset;
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
        port = master_port + port_offset
        if rank == 0:
            tracker = RabitTracker(addr, world, port=port, port_end=port + 1,
                                   print_fn=lambda m: None)
            tracker.start(world)
    args = dict(rabit_tracker_uri=addr, rabit_tracker_port=port, rabit_task_id=rank,
                rabit_world_size=world, DMLC_WORKER_CONNECT_RETRY=30)
    if "rabit_device" not in params:
        params["rabit_device"] = local_rank
    args.update(params)
    rabit.init(lib=lib, **args)
    assert rabit.get_world_size() == world, "rabit world size differs from torchrun's"
    return TorchrunContext(rank, world, local_rank, tracker)
