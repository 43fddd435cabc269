"""Replay a launch-bound per-iteration device closure as one hipGraph.

A training step of a small or deep model is a few hundred short kernels (forward, backward,
zeroing the gradient buckets); on MI355X each costs a few microseconds of host launch time,
often more than the kernel itself.  `GraphedStep` captures the closure once into a hipGraph
(`torch.cuda.CUDAGraph` is hipGraph on ROCm) and replays it with one launch per step.

The collectives stay outside the graph on purpose: a rabit collective is host logic as much as
device work (sequence numbers, the result log, consensus, recovery and replay after a failure),
so `GradientBuckets.reduce()` runs after the replay, on the same stream, exactly as in an eager
step.  The graph ends by writing the gradients into the bucket views (one multi-tensor copy), so
the collective reads them where they are.

    def compute_loss_and_grads():
        loss = loss_fn(model(xs_static), ys_static)
        buckets.backward(loss)     # functional gradients into the buckets (graph-exact)
        return loss

    step = GraphedStep(compute_loss_and_grads)  # static inputs: copy new data in
    for it in loop:
        xs_static.copy_(next_batch)
        loss = step()              # warm-up runs eagerly, then capture + replay, then replay
        buckets.reduce()           # fault-tolerant allreduce of the gradient buckets
        optimizer_update()

Every call executes the closure exactly once (warm-up calls run it eagerly; the capturing call
replays right after capturing), so a job does the same work whether or not it is graphed.
Measured on MI355X (profiles/r1_graphs/): the graphed runs of tools/graph_steps.py and
examples/dp_train.py (3 ranks) end with weights bit-identical to the eager runs.

Produce the gradients with `GradientBuckets.backward(loss)` (torch.autograd.grad + one copy into
the buckets) inside the closure, not with `loss.backward()`: on this PyTorch-ROCm build a
captured *accumulating* backward pass replays exactly once and then yields wrong gradients for
some shapes; the culprit is the column reduction of the bias gradient (torch.sum(x, 0) on
[512, 1024] replays wrongly from its second replay on: tools/graph_reduce_check.py).

With workers killed and restarted, graphed runs of models with `nn.Linear` biases could end
with different weights: the column reduction again, on a survivor's replay after the recovery.
`graph_safe_linear(model)` computes bias gradients as GEMVs; with it (or without biases) every
failure case tried is bit-identical to the clean eager run (tools/graph_check.py).
"""
from __future__ import annotations

from typing import Any, Callable, Optional


class GraphedStep:
    def __init__(self, fn: Callable[[], Any], warmup: int = 3, enabled: bool = True):
        """fn: the per-iteration device work.  It must read its inputs from tensors whose
        storage stays the same between calls (copy new batches into them) and may return
        tensors (or a structure of them); the returned objects are the graph's static outputs,
        overwritten by every replay.  warmup: eager calls before capturing (autograd and the
        allocator need them; they run on a side stream as capture requires)."""
        self.fn = fn
        self.warmup = max(1, int(warmup))
        self.enabled = enabled
        self.calls = 0
        self.graph = None
        self.out: Optional[Any] = None
        self._side = None

    @property
    def captured(self) -> bool:
        return self.graph is not None

    def __call__(self) -> Any:
        import torch

        self.calls += 1
        if not self.enabled or not torch.cuda.is_available():
            return self.fn()
        if self.graph is not None:
            self.graph.replay()
            return self.out
        cur = torch.cuda.current_stream()
        if self._side is None:
            self._side = torch.cuda.Stream()
        self._side.wait_stream(cur)
        if self.calls <= self.warmup:
            with torch.cuda.stream(self._side):
                out = self.fn()
            cur.wait_stream(self._side)
            return out
        return self._capture(cur)

    def _capture(self, cur) -> Any:
        import torch

        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=self._side):
            self.out = self.fn()
        self.graph = g
        # capturing recorded the kernels without running them: this call's work is the replay
        g.replay()
        return self.out


def _linear_fn():
    import torch

    class _GraphSafeLinear(torch.autograd.Function):
        """nn.Linear with the bias gradient as a GEMV (dY^T @ 1) instead of a column reduction"""

        @staticmethod
        def forward(ctx, x, w, b):
            ctx.save_for_backward(x, w)
            ctx.has_bias = b is not None
            return torch.nn.functional.linear(x, w, b)

        @staticmethod
        def backward(ctx, gy):
            x, w = ctx.saved_tensors
            gy2 = gy.reshape(-1, gy.shape[-1])
            x2 = x.reshape(-1, x.shape[-1])
            gx = (gy2 @ w).view(x.shape) if ctx.needs_input_grad[0] else None
            gw = gy2.t() @ x2
            gb = None
            if ctx.has_bias:
                ones = torch.ones(gy2.shape[0], dtype=gy.dtype, device=gy.device)
                gb = torch.mv(gy2.t(), ones)
            return gx, gw, gb

    return _GraphSafeLinear


def graph_safe_linear(model):
    """Make every nn.Linear of `model` compute its bias gradient with a GEMV instead of the
    column reduction torch uses (which this PyTorch-ROCm build replays wrongly from a hipGraph
    for some shapes, profiles/r1_graphs/).  Same forward; the weight and input gradients are the
    same GEMMs.  Apply it to the eager and the graphed model alike when their results are
    compared bit for bit (the bias gradient's summation order differs from torch's)."""
    import torch

    fn = _linear_fn()
    for m in model.modules():
        if isinstance(m, torch.nn.Linear):
            m.forward = (lambda mod: (lambda x: fn.apply(x, mod.weight, mod.bias)))(m)
    return model
