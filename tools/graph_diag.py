"""Gradients of one step, eager vs GraphedStep replay, same weights and data (no update):
which configuration makes repeated replays of a captured forward+backward exact."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rabit_amd.parallel import GraphedStep  # noqa: E402


def main(layers, hidden, batch, variant):
    dev = torch.device("cuda", 0)
    if variant == "rocblas":
        torch.backends.cuda.preferred_blas_library("cublas")
    else:
        torch.backends.cuda.preferred_blas_library("default")
    torch.manual_seed(0)
    mods = []
    for _ in range(layers):
        mods += [torch.nn.Linear(hidden, hidden), torch.nn.Tanh()]
    model = torch.nn.Sequential(*mods, torch.nn.Linear(hidden, 1)).to(dev)
    params = list(model.parameters())
    for p in params:
        p.grad = torch.zeros_like(p)
    xs = torch.randn(batch, hidden, device=dev)
    ys = torch.randn(batch, 1, device=dev)

    def compute():
        if variant == "autograd_grad":
            loss = torch.nn.functional.mse_loss(model(xs), ys)
            gs = torch.autograd.grad(loss, params)
            for p, g in zip(params, gs):
                p.grad.copy_(g)
            return loss
        for p in params:
            p.grad.zero_()
        loss = torch.nn.functional.mse_loss(model(xs), ys)
        loss.backward()
        return loss

    compute()
    torch.cuda.synchronize()
    g_eager = torch.cat([p.grad.reshape(-1) for p in params]).clone()
    st = GraphedStep(compute, warmup=11 if variant == "warmup11" else 3)
    res = []
    for i in range(st.warmup + 4):
        loss = st()
        torch.cuda.synchronize()
        g = torch.cat([p.grad.reshape(-1) for p in params])
        res.append(float((g - g_eager).abs().max()))
    per = {}
    off = 0
    for i, p in enumerate(params):
        k = p.numel()
        e = float((g[off:off + k] - g_eager[off:off + k]).abs().max())
        if e > 0:
            per["p%d%s" % (i, list(p.shape))] = e
        off += k
    return {"layers": layers, "hidden": hidden, "batch": batch, "variant": variant,
            "bad_params_last": per,
            "graph_call_maxdiff": res, "gmax": float(g_eager.abs().max()),
            "ratio_last": float((g / g_eager.where(g_eager.abs() > 1e-6, torch.ones_like(g_eager)))
                                .median())}


for v in sys.argv[1:] or ["default", "rocblas", "autograd_grad", "warmup11"]:
    for cfg in [(4, 2048, 1024), (2, 1024, 512)]:
        try:
            print(json.dumps(main(*cfg, v)), flush=True)
        except Exception as e:  # noqa: BLE001
            print(json.dumps({"variant": v, "cfg": cfg, "error": repr(e)[:300]}), flush=True)
