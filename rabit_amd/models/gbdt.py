"""Histogram gradient-boosted trees (the XGBoost "hist" workload that rabit was built for).

Each rank holds a row shard.  Per tree level every rank builds (node, feature, bin) gradient /
hessian histograms of its rows (one scatter-add on the device), a single rabit allreduce sums
them across ranks, and every rank runs the same split search on the same numbers, so the
trees are identical everywhere.  Trees are the checkpointed global state: a restarted worker
reloads them, recomputes its margins, and replays the histogram reductions it missed.
"""
from __future__ import annotations

from typing import List

from .. import core as rabit
from ..parallel.data_parallel import FaultTolerantLoop


class HistGBDT:
    def __init__(self, n_trees: int = 10, max_depth: int = 4, n_bins: int = 64,
                 learning_rate: float = 0.3, l2: float = 1.0, min_child_weight: float = 1e-3,
                 objective: str = "binary"):
        assert objective in ("binary", "regression")
        self.n_trees, self.depth, self.n_bins = n_trees, max_depth, n_bins
        self.lr, self.l2, self.mcw, self.objective = learning_rate, l2, min_child_weight, objective
        self.trees: List[dict] = []
        self.lo = self.hi = None
        self.base = 0.0
        self.hist_allreduce_bytes = 0

    # ---------------------------------------------------------------- binning
    def _fit_bins(self, x):
        import torch

        lo = x.min(dim=0).values.double().contiguous()
        hi = x.max(dim=0).values.double().contiguous()
        rabit.allreduce(lo, rabit.MIN)
        rabit.allreduce(hi, rabit.MAX)
        self.lo, self.hi = lo.cpu(), hi.cpu()

    def _bin(self, x):
        import torch

        lo, hi = self.lo.to(x.device), self.hi.to(x.device)
        span = torch.where(hi > lo, hi - lo, torch.ones_like(hi))
        b = ((x.double() - lo) / span * self.n_bins).floor().clamp_(0, self.n_bins - 1)
        return b.to(torch.int64)

    # ---------------------------------------------------------------- objective
    def _grad_hess(self, margin, y):
        import torch

        if self.objective == "binary":
            p = torch.sigmoid(margin)
            return p - y, (p * (1 - p)).clamp_min(1e-16)
        return margin - y, torch.ones_like(margin)

    # ---------------------------------------------------------------- one tree
    def _grow(self, xb, g, h):
        import torch

        n, d = xb.shape
        nb, lam = self.n_bins, self.l2
        n_nodes = 2 ** (self.depth + 1) - 1
        feature = torch.full((n_nodes,), -1, dtype=torch.int64)
        thresh = torch.zeros(n_nodes, dtype=torch.int64)
        node = torch.zeros(n, dtype=torch.int64, device=xb.device)
        is_leaf = torch.zeros(n_nodes, dtype=torch.bool)
        for level in range(self.depth):
            first, count = 2 ** level - 1, 2 ** level
            local = node - first
            active = (local >= 0) & (local < count)
            rows = active.nonzero(as_tuple=True)[0]
            hist = torch.zeros(count * d * nb * 2, dtype=torch.float64, device=xb.device)
            if rows.numel() > 0:
                ln = local[rows].unsqueeze(1)
                base = (ln * d + torch.arange(d, device=xb.device).unsqueeze(0)) * nb + xb[rows]
                idx = (base * 2).reshape(-1)
                hist.index_add_(0, idx, g[rows].double().repeat_interleave(d))
                hist.index_add_(0, idx + 1, h[rows].double().repeat_interleave(d))
            rabit.allreduce(hist, rabit.SUM)  # the rabit workload
            self.hist_allreduce_bytes += hist.numel() * 8
            H = hist.view(count, d, nb, 2).cpu()
            cum = H.cumsum(dim=2)
            GL, HL = cum[..., 0], cum[..., 1]
            Gt, Ht = cum[:, 0, -1, 0], cum[:, 0, -1, 1]
            GR, HR = Gt[:, None, None] - GL, Ht[:, None, None] - HL
            parent = (Gt ** 2 / (Ht + lam))[:, None, None]
            gain = GL ** 2 / (HL + lam) + GR ** 2 / (HR + lam) - parent
            ok = (HL >= self.mcw) & (HR >= self.mcw)
            ok[..., nb - 1] = False
            gain = torch.where(ok, gain, torch.full_like(gain, -1.0))
            best = gain.view(count, -1).max(dim=1)
            for j in range(count):
                nid = first + j
                if is_leaf[nid] or Ht[j] <= 0:
                    is_leaf[nid] = True
                    continue
                if best.values[j] <= 1e-12:
                    is_leaf[nid] = True
                    continue
                f, b = divmod(int(best.indices[j]), nb)
                feature[nid], thresh[nid] = f, b
            # route active rows of split nodes to their children
            nid_rows = node[rows]
            f_rows = feature.to(xb.device)[nid_rows]
            split = f_rows >= 0
            if split.any():
                r2 = rows[split]
                fr = f_rows[split]
                go_left = xb[r2, fr] <= thresh.to(xb.device)[node[r2]]
                node[r2] = torch.where(go_left, 2 * node[r2] + 1, 2 * node[r2] + 2)
            for j in range(count):
                nid = first + j
                if feature[nid] < 0:
                    is_leaf[nid] = True
                    for c in (2 * nid + 1, 2 * nid + 2):
                        is_leaf[c] = True  # unreachable children
        # leaf values from global (G, H) per node
        gh = torch.zeros(n_nodes * 2, dtype=torch.float64, device=xb.device)
        gh.index_add_(0, node * 2, g.double())
        gh.index_add_(0, node * 2 + 1, h.double())
        rabit.allreduce(gh, rabit.SUM)
        gh = gh.view(n_nodes, 2).cpu()
        value = -self.lr * gh[:, 0] / (gh[:, 1] + lam)
        return {"feature": feature, "thresh": thresh, "value": value}

    def _tree_predict(self, tree, xb):
        import torch

        node = torch.zeros(xb.shape[0], dtype=torch.int64, device=xb.device)
        feature = tree["feature"].to(xb.device)
        thresh = tree["thresh"].to(xb.device)
        for _ in range(self.depth):
            f = feature[node]
            split = f >= 0
            fcl = f.clamp_min(0)
            left = xb.gather(1, fcl.unsqueeze(1)).squeeze(1) <= thresh[node]
            child = torch.where(left, 2 * node + 1, 2 * node + 2)
            node = torch.where(split, child, node)
        return tree["value"].to(xb.device)[node]

    # ---------------------------------------------------------------- API
    def fit(self, x, y):
        """x: local rows [n, d], y: [n] (0/1 for binary)."""
        import torch

        def get_state():
            return {"trees": self.trees, "base": self.base, "lo": self.lo, "hi": self.hi}

        def set_state(s):
            self.trees = list(s["trees"])
            self.base, self.lo, self.hi = s["base"], s["lo"], s["hi"]

        loop = FaultTolerantLoop(get_state, set_state, 1)
        y = y.double()
        if not loop.load():
            # setup collectives run once, in version 0; their results are checkpointed
            self._fit_bins(x)
            stats = torch.stack([y.sum(), torch.tensor(float(y.numel()), device=y.device,
                                                       dtype=torch.float64)]).contiguous()
            rabit.allreduce(stats, rabit.SUM)
            mean = float(stats[0] / stats[1])
            if self.objective == "binary":
                mean = min(max(mean, 1e-6), 1 - 1e-6)
                self.base = float(torch.log(torch.tensor(mean / (1 - mean))))
            else:
                self.base = mean
        xb = self._bin(x)
        margin = torch.full_like(y, self.base)
        for it in loop.iterations(self.n_trees):
            if it == loop.start and self.trees:
                margin = torch.full_like(y, self.base)
                for t in self.trees:
                    margin += self._tree_predict(t, xb)
            g, h = self._grad_hess(margin, y)
            tree = self._grow(xb, g, h)
            self.trees.append(tree)
            margin = margin + self._tree_predict(tree, xb)
            loop.step_done(it)
        return self

    def decision_function(self, x):
        import torch

        xb = self._bin(x)
        m = torch.full((x.shape[0],), self.base, dtype=torch.float64, device=x.device)
        for t in self.trees:
            m += self._tree_predict(t, xb)
        return m

    def predict_proba(self, x):
        import torch

        return torch.sigmoid(self.decision_function(x))
