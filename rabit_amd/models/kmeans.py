"""Distributed k-means (rabit's canonical example workload).

Each rank holds a shard of the points (torch tensor on CPU or HBM).  Per iteration the
per-cluster statistics [sum of points | count] are produced by a *lazy prepare function* and
allreduced: after a failure, a restarted worker replays the reduced statistics of the
iterations it missed from its peers without recomputing its assignments.  Centroids are the
global checkpointed state.
"""
from __future__ import annotations

from typing import Optional

from .. import core as rabit
from ..parallel.data_parallel import FaultTolerantLoop


class KMeans:
    def __init__(self, k: int, n_iter: int = 10, seed: int = 0, checkpoint_every: int = 1):
        self.k, self.n_iter, self.seed, self.every = k, n_iter, seed, checkpoint_every
        self.centroids = None
        self.prepare_calls = 0
        self.inertia_: Optional[float] = None

    def _init_centroids(self, x):
        """Distributed farthest-point seeding: a random first centre from rank 0, then
        repeatedly the global point farthest from the chosen centres (one allgather of the
        per-rank best distance and one broadcast of the winner's point per centre)."""
        import torch

        d = x.shape[1]
        c = torch.zeros(self.k, d, dtype=x.dtype, device=x.device)
        if rabit.get_rank() == 0:
            g = torch.Generator(device="cpu").manual_seed(self.seed)
            c[0] = x[int(torch.randint(0, x.shape[0], (1,), generator=g))]
        c[0:1] = rabit.broadcast_tensor(c[0:1].contiguous(), 0)
        for j in range(1, self.k):
            dist = torch.cdist(x, c[:j]).min(dim=1).values
            best = int(dist.argmax()) if x.shape[0] > 0 else 0
            val = float(dist[best]) if x.shape[0] > 0 else -1.0
            vals = rabit.allgather(torch.tensor([val], dtype=torch.float64))
            owner = int(vals.argmax())
            pt = x[best:best + 1].clone() if rabit.get_rank() == owner else torch.zeros(
                1, d, dtype=x.dtype, device=x.device)
            c[j:j + 1] = rabit.broadcast_tensor(pt.contiguous(), owner)
        return c

    def fit(self, x):
        """x: local shard [n_local, d] (float32/float64); returns the global centroids."""
        import torch

        x = x.contiguous()
        state = {}

        def get_state():
            return self.centroids.detach().cpu().numpy()

        def set_state(s):
            state["resumed"] = True
            self.centroids = torch.as_tensor(s, device=x.device)

        loop = FaultTolerantLoop(get_state, set_state, self.every)
        k, d = self.k, x.shape[1]
        for it in loop.iterations(self.n_iter):
            if self.centroids is None:
                self.centroids = self._init_centroids(x)
            stats = torch.zeros(k, d + 1, dtype=torch.float64, device=x.device)

            def prepare(buf):
                self.prepare_calls += 1
                assign = torch.cdist(x, self.centroids.to(x.dtype)).argmin(dim=1)
                buf[:, :d].index_add_(0, assign, x.double())
                buf[:, d].index_add_(0, assign, torch.ones_like(assign, dtype=torch.float64))

            rabit.allreduce(stats.view(-1), rabit.SUM, prepare_fun=lambda _b: prepare(stats))
            counts = stats[:, d:d + 1]
            new = torch.where(counts > 0, stats[:, :d] / counts.clamp(min=1),
                              self.centroids.double())
            self.centroids = new.to(x.dtype)
            loop.step_done(it)
        # final inertia (one more collective)
        dist = torch.cdist(x, self.centroids).min(dim=1).values.pow(2).sum().double()
        inertia = dist.reshape(1).contiguous()
        rabit.allreduce(inertia, rabit.SUM)
        self.inertia_ = float(inertia.item())
        return self.centroids

    def predict(self, x):
        import torch

        return torch.cdist(x, self.centroids.to(x.dtype)).argmin(dim=1)
