"""Distributed linear / logistic regression with L-BFGS.

Data-parallel full-batch optimisation: every rank computes the loss and gradient of its shard,
one allreduce sums [loss | grad] (a single collective per evaluation), and because every rank
then runs the same L-BFGS update on identical numbers the model stays identical everywhere —
the "global model" rabit checkpoints.  Works on CPU tensors and HBM tensors.
"""
from __future__ import annotations

from .. import core as rabit
from ..parallel.data_parallel import FaultTolerantLoop


class LinearModel:
    def __init__(self, n_features: int, loss: str = "logistic", l2: float = 1e-4,
                 n_iter: int = 20, lbfgs_history: int = 10, device=None, dtype=None):
        import torch

        assert loss in ("logistic", "squared")
        self.loss, self.l2, self.n_iter, self.hist = loss, l2, n_iter, lbfgs_history
        self.device = device or torch.device("cpu")
        self.dtype = dtype or torch.float64
        self.w = torch.zeros(n_features + 1, dtype=self.dtype, device=self.device)
        self.history = []

    def _local_objective(self, x, y, w):
        import torch

        z = x @ w[:-1] + w[-1]
        if self.loss == "logistic":
            return torch.nn.functional.softplus(-y * z).sum()  # y in {-1, +1}
        return 0.5 * ((z - y) ** 2).sum()

    def _global_loss_grad(self, x, y, n_total, w):
        import torch

        w = w.detach().requires_grad_(True)
        f = self._local_objective(x, y, w)
        (g,) = torch.autograd.grad(f, w)
        buf = torch.cat([f.detach().reshape(1), g]).contiguous()
        rabit.allreduce(buf, rabit.SUM)
        loss = buf[0] / n_total + 0.5 * self.l2 * (w.detach()[:-1] ** 2).sum()
        grad = buf[1:] / n_total
        grad[:-1] += self.l2 * w.detach()[:-1]
        return loss, grad

    def fit(self, x, y):
        """x: local shard [n, d], y: [n] (+-1 for logistic).  Returns the global weights."""
        import torch

        x = x.to(self.device, self.dtype)
        y = y.to(self.device, self.dtype)
        w_param = torch.nn.Parameter(self.w.clone())
        opt = torch.optim.LBFGS([w_param], lr=1.0, max_iter=1, history_size=self.hist,
                                line_search_fn="strong_wolfe")
        meta = {}

        def closure():
            loss, grad = self._global_loss_grad(x, y, meta["n_total"], w_param)
            w_param.grad = grad.to(w_param.dtype)
            return loss

        def get_state():
            return {"w": w_param.detach().cpu().numpy(), "opt": opt.state_dict(),
                    "n_total": meta["n_total"], "history": self.history}

        def set_state(s):
            with torch.no_grad():
                w_param.copy_(torch.as_tensor(s["w"]).to(w_param))
            opt.load_state_dict(s["opt"])
            meta["n_total"] = s["n_total"]
            self.history = list(s["history"])

        loop = FaultTolerantLoop(get_state, set_state, 1)
        if not loop.load():
            meta["n_total"] = rabit.allreduce(
                torch.tensor([float(x.shape[0])], dtype=torch.float64), rabit.SUM).item()
        for it in loop.iterations(self.n_iter):
            loss = opt.step(closure)
            self.history.append(float(loss))
            loop.step_done(it)
        self.w = w_param.detach()
        return self.w

    def decision_function(self, x):
        x = x.to(self.device, self.dtype)
        return x @ self.w[:-1] + self.w[-1]

    def predict(self, x):
        import torch

        z = self.decision_function(x)
        return torch.sign(z) if self.loss == "logistic" else z
