"""Step time of a launch-bound data-parallel training step, eager vs GraphedStep (hipGraph).

One rank (world 1, the engine's world-1 short-circuit off so the gradient bucket goes through
the robust engine's device path).  The step is dp_train.py's: zero the HBM gradient bucket,
forward + backward of a deep, narrow MLP (many short kernels), fault-tolerant bucket
allreduce, fused multi-tensor SGD update.  Prints one JSON line.

    python tools/graph_probe.py --layers 16 --hidden 512 --batch 256
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import rabit_amd as rabit  # noqa: E402
from rabit_amd.parallel import GradientBuckets, GraphedStep, graph_safe_linear  # noqa: E402


def build(args, dev):
    torch.manual_seed(0)
    layers = []
    for _ in range(args.layers):
        layers += [torch.nn.Linear(args.hidden, args.hidden), torch.nn.Tanh()]
    model = torch.nn.Sequential(*layers, torch.nn.Linear(args.hidden, 1)).to(dev)
    if args.safe_linear:
        graph_safe_linear(model)
    buckets = GradientBuckets(model.parameters(), bucket_mb=256)
    return model, buckets


def run(args, dev, graphed):
    model, buckets = build(args, dev)
    params = list(model.parameters())
    xs = torch.randn(args.batch, args.hidden, device=dev)
    ys = torch.randn(args.batch, 1, device=dev)

    def compute():
        loss = torch.nn.functional.mse_loss(model(xs), ys)
        buckets.backward(loss)
        return loss

    step_fn = GraphedStep(compute) if graphed else compute
    grads = [p.grad for p in params]

    def step():
        loss = step_fn()
        buckets.reduce()
        with torch.no_grad():
            torch._foreach_add_(params, grads, alpha=-1e-3)
        return loss

    for _ in range(args.warmup):
        step()
    rabit.checkpoint(None)  # clears the HBM result log
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.steps
    loss = float(loss.item())  # a graph's output is overwritten by the next replay
    # the pure GPU time of one step (one replayed graph + collective), from device events
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(args.steps):
        step()
    ev1.record()
    torch.cuda.synchronize()
    w = torch.cat([p.detach().reshape(-1) for p in params])
    info = {"captured": bool(getattr(step_fn, "captured", False))}
    return dt, ev0.elapsed_time(ev1) / args.steps * 1e-3, loss, w, info


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=16)
    ap.add_argument("--hidden", type=int, default=512)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--safe-linear", type=int, default=0,
                    help="bias gradients as GEMVs in both runs (graph_safe_linear)")
    args = ap.parse_args()
    rabit.init([], lib="standard", rabit_world1_fastpath=0)
    dev = torch.device("cuda", 0)
    t_eager, g_eager, l_eager, w_eager, _ = run(args, dev, False)
    t_graph, g_graph, l_graph, w_graph, info = run(args, dev, True)
    rec = {"probe": "graphed_step", "safe_linear": args.safe_linear, "layers": args.layers, "hidden": args.hidden,
           "batch": args.batch, "steps": args.steps,
           "eager_us": round(t_eager * 1e6, 1), "graphed_us": round(t_graph * 1e6, 1),
           "speedup": round(t_eager / t_graph, 2),
           "eager_loop_events_us": round(g_eager * 1e6, 1),
           "graphed_loop_events_us": round(g_graph * 1e6, 1),
           "identical_weights": bool(torch.equal(w_eager, w_graph)),
           "graph": info,
           "loss": [l_eager, l_graph],
           "device_ops": rabit.stats().get("n_device_ops", 0)}
    print(json.dumps(rec), flush=True)
    rabit.finalize()


if __name__ == "__main__":
    main()
