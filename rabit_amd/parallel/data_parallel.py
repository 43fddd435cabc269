"""Bucketed gradient allreduce and a fault-tolerant iteration loop."""
from __future__ import annotations

from typing import Callable, Dict, Iterable, List, Optional

import numpy as np

from .. import core as rabit


class GradientBuckets:
    """Flatten a model's gradients into a few large contiguous buckets.

    Every parameter's `.grad` becomes a view into a bucket, so autograd accumulates directly
    into the buffers that are reduced (no pack/unpack copies).  `reduce()` issues one
    collective per bucket: large messages are what the xGMI ring needs to reach bandwidth
    (SURVEY §5.8), and with 288 GB of HBM a 256 MB bucket costs nothing.  On HBM the
    averaging (x 1/world) runs in the fused lazy-prepare kernel of the same call, so it is
    skipped together with the reduction when the result is replayed after a failure.
    """

    def __init__(self, params: Iterable, bucket_mb: float = 256.0, average: bool = True,
                 symmetric: bool = False):
        import torch

        self.params = [p for p in params if p.requires_grad]
        self.average = average
        # symmetric=True: HBM buckets come from the engine's symmetric heap (init with
        # rabit_device_symmetric_heap), so the direct transport reduces them in place without a
        # staging copy; the heap is uncached, which the gradient-producing kernels also see
        self.symmetric = symmetric
        cap = max(1, int(bucket_mb * (1 << 20)))
        self.buckets: List["torch.Tensor"] = []
        self._groups: List[List] = []
        groups: Dict[tuple, List] = {}
        for p in self.params:  # bucket per (device, dtype)
            groups.setdefault((p.device, p.dtype), []).append(p)
        for (dev, dtype), plist in groups.items():
            cur, size = [], 0
            esz = torch.empty((), dtype=dtype).element_size()
            for p in plist:
                if cur and (size + p.numel()) * esz > cap:
                    self._make_bucket(cur, size, dev, dtype)
                    cur, size = [], 0
                cur.append(p)
                size += p.numel()
            if cur:
                self._make_bucket(cur, size, dev, dtype)

    def _make_bucket(self, plist, size, dev, dtype):
        import torch

        if self.symmetric and dev.type == "cuda":
            flat = rabit.symmetric_empty(size, dtype)
            flat.zero_()
        else:
            flat = torch.zeros(size, dtype=dtype, device=dev)
        off = 0
        for p in plist:
            n = p.numel()
            if p.grad is not None:
                flat[off:off + n].copy_(p.grad.reshape(-1))
            p.grad = flat[off:off + n].view_as(p)
            off += n
        self.buckets.append(flat)
        self._groups.append(plist)

    def zero_grad(self):
        for b in self.buckets:
            b.zero_()

    def backward(self, loss):
        """Write d(loss)/d(param) into the buckets, overwriting (no zero_grad needed).

        Functional (`torch.autograd.grad`, then one multi-tensor copy into the bucket views)
        rather than `loss.backward()`'s accumulation into `.grad`: the same gradient kernels
        run, so the values are identical, and it stays exact when the step is replayed as a
        hipGraph.  Accumulating backward passes captured in a graph gave wrong bias gradients
        from the second replay on for some shapes on this PyTorch-ROCm build
        (tools/graph_diag.py, profiles/r1_graphs/)."""
        import torch

        grads = torch.autograd.grad(loss, self.params, allow_unused=True)
        dst, src = [], []
        for p, g in zip(self.params, grads):
            if g is None:
                p.grad.zero_()
            else:
                dst.append(p.grad)
                src.append(g)
        if dst:
            torch._foreach_copy_(dst, src)

    def reduce(self, op: int = rabit.SUM, graphable: bool = False):
        """Allreduce every bucket (in place); returns the buckets.

        graphable=True: HBM buckets go through `rabit.allreduce_graphable` (a bare in-place
        allreduce on the current stream over RCCL or the direct transport, no host
        synchronisation), so the call can sit inside a captured hipGraph with the rest of the
        step.  Non-fault-tolerant engines only (init(lib="base")); averaging is one `mul_` on the
        same stream, captured as well.  Limits: a replayed graph has no failure probe (a dead
        peer stalls replay() until the direct barriers' deadline, or hangs RCCL; this is the base
        engine's contract).  Multi-rank capture over the direct transport is tested
        (tests/scripts/graph_direct.py: replayed buckets equal world x the local gradient); a
        captured multi-rank RCCL reduction has only run with a one-rank communicator so far."""
        world = rabit.get_world_size()
        if graphable:
            for b in self.buckets:
                if not b.is_cuda:
                    raise TypeError("graphable reduce needs HBM buckets")
                rabit.allreduce_graphable(b, op)
                if self.average and op == rabit.SUM and world > 1:
                    b.mul_(1.0 / world)
            return self.buckets
        for b in self.buckets:
            if b.is_cuda and self.average and op == rabit.SUM and world > 1:
                rabit.allreduce_prepared(b, b, op, rabit.PREP_SCALE, 1.0 / world)
            else:
                rabit.allreduce(b, op)
                if self.average and op == rabit.SUM and world > 1:
                    b.mul_(1.0 / world)
        return self.buckets


class FaultTolerantLoop:
    """Iterative job in rabit's recovery model.

        loop = FaultTolerantLoop(get_state, set_state, checkpoint_every=1)
        for it in loop.iterations(n_iter):
            ...collectives...
            loop.step_done(it)

    `get_state()` returns a picklable global state (identical on all ranks), `set_state` loads
    it; a restarted worker resumes from the last checkpoint and replays missed collectives.
    """

    def __init__(self, get_state: Callable[[], object], set_state: Callable[[object], None],
                 checkpoint_every: int = 1, get_local: Optional[Callable[[], object]] = None,
                 set_local: Optional[Callable[[object], None]] = None):
        self.get_state, self.set_state = get_state, set_state
        self.get_local, self.set_local = get_local, set_local
        self.every = max(1, checkpoint_every)
        self.start = 0
        self.loaded = False
        self.resumed = False

    def load(self) -> bool:
        """Load the last checkpoint.  Must precede every collective of the job: a restarted
        worker replays collectives by (version, seqno), so setup collectives belong after
        this call and only when not resumed (their results are part of the state).
        Returns True when the state was restored."""
        if self.loaded:
            return self.resumed
        self.loaded = True
        if self.get_local is not None:
            version, state, local = rabit.load_checkpoint(with_local=True)
            if version > 0:
                self.set_local(local)
        else:
            version, state = rabit.load_checkpoint()
        if version > 0:
            self.set_state(state["state"])
            self.start = int(state["next_iter"])
            self.resumed = True
        return self.resumed

    def iterations(self, n_iter: int):
        self.load()
        for it in range(self.start, n_iter):
            yield it

    def step_done(self, it: int):
        if (it + 1) % self.every == 0:
            g = {"state": self.get_state(), "next_iter": it + 1}
            if self.get_local is not None:
                rabit.checkpoint(g, self.get_local())
            else:
                rabit.checkpoint(g)


def shard(n: int, rank: int, world: int):
    """[begin, end) of an even split of n items."""
    per = (n + world - 1) // world
    return min(n, rank * per), min(n, (rank + 1) * per)


def global_mean(x: np.ndarray) -> np.ndarray:
    """Mean over ranks (host arrays)."""
    total = rabit.allreduce(np.asarray(x, dtype=np.float64).copy(), rabit.SUM)
    return total / rabit.get_world_size()
