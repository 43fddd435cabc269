"""Single process, no collectives: dp_train's model trained eagerly and through GraphedStep;
reports the first step whose weights differ (-1: bit-identical for all steps)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rabit_amd.parallel import GradientBuckets, GraphedStep  # noqa: E402


def train(graph, hidden, layers, rows, steps=12, det=True):
    torch.use_deterministic_algorithms(det, warn_only=True)
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(1234)
    X = torch.randn(rows, 32, generator=g).to(dev)
    y = torch.randn(rows, 1, generator=g).to(dev)
    torch.manual_seed(0)
    mods = [torch.nn.Linear(32, hidden), torch.nn.Tanh()]
    for _ in range(layers - 1):
        mods += [torch.nn.Linear(hidden, hidden), torch.nn.Tanh()]
    model = torch.nn.Sequential(*mods, torch.nn.Linear(hidden, 1)).to(dev)
    buckets = GradientBuckets(model.parameters(), bucket_mb=1)

    def compute():
        loss = torch.nn.functional.mse_loss(model(X), y)
        buckets.backward(loss)
        return loss

    fn = GraphedStep(compute) if graph else compute
    hist = []
    for _ in range(steps):
        fn()
        with torch.no_grad():
            for p in model.parameters():
                p.add_(p.grad, alpha=-0.05)
        hist.append(torch.cat([p.detach().reshape(-1) for p in model.parameters()]).clone())
    torch.cuda.synchronize()
    return hist, getattr(fn, "captured", False)


for hidden, layers, rows in [(256, 6, 2000), (1024, 3, 2000), (512, 1, 2000), (256, 6, 512)]:
    for det in (True, False):
        ref, _ = train(False, hidden, layers, rows, det=det)
        hist, cap = train(True, hidden, layers, rows, det=det)
        first = next((i for i, (a, b) in enumerate(zip(ref, hist)) if not torch.equal(a, b)), -1)
        print(json.dumps({"hidden": hidden, "layers": layers, "rows": rows, "det": det,
                          "captured": cap, "first_diff_step": first}), flush=True)
