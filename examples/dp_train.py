"""Fault-tolerant data-parallel training of an MLP on HBM: the whole xrabit stack in one job.

Each rank trains on its own shard of a synthetic regression set.  Per iteration:
forward/backward on the GPU -> GradientBuckets.reduce() (one fused average-allreduce per HBM
bucket over the device transports) -> SGD step -> checkpoint_tensors() every `--ckpt` steps
(HBM snapshot + async pinned mirror).  A worker that dies (mock=rank,version,seq,trial with
lib=mock, or a real crash under the launcher) is restarted, reloads the last checkpoint from
the survivors, and replays the gradient allreduces it missed from their HBM result logs — its
own gradients for those steps are never needed — so the final weights are bit-identical to a
run without failures.  Rank 0 prints a hash of the final weights.

    python -m rabit_amd.launcher -n 3 --num-attempt 3 -- python examples/dp_train.py \
        --steps 12 lib=mock mock=1,2,1,0
"""
import argparse
import hashlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import rabit_amd as rabit  # noqa: E402
from rabit_amd.parallel.data_parallel import GradientBuckets, shard  # noqa: E402
from rabit_amd.parallel.graphs import GraphedStep, graph_safe_linear  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=12)
    ap.add_argument("--ckpt", type=int, default=3, help="checkpoint every this many steps")
    ap.add_argument("--hidden", type=int, default=512)
    ap.add_argument("--rows", type=int, default=6000)
    ap.add_argument("--lr", type=float, default=0.05)
    ap.add_argument("--bucket-mb", type=float, default=0.25)
    ap.add_argument("--graph", type=int, default=0,
                    help="replay forward+backward as one hipGraph (GraphedStep); bit-identical")
    ap.add_argument("--layers", type=int, default=1, help="hidden layers of the MLP")
    ap.add_argument("--bias", type=int, default=1, help="0: bias-free hidden layers")
    ap.add_argument("--safe-linear", type=int, default=0,
                    help="bias gradients as GEMVs (graph_safe_linear); use with --graph")
    ap.add_argument("--trace-steps", type=int, default=0,
                    help="print a digest of the local and the reduced gradients every step")
    args, rest = ap.parse_known_args()
    lib = "standard"
    params = []
    for a in rest:
        if a.startswith("lib="):
            lib = a[4:]
        else:
            params.append(a)
    ngpu = torch.cuda.device_count()
    rank_hint = int(os.environ.get("DMLC_TASK_ID", os.environ.get("RANK", "0")))
    gpu = rank_hint % max(ngpu, 1)
    rabit.init(params, lib=lib, rabit_device=gpu)
    rank, world = rabit.get_rank(), rabit.get_world_size()
    dev = torch.device("cuda", gpu) if ngpu else torch.device("cpu")
    torch.use_deterministic_algorithms(True, warn_only=True)

    # identical initial weights and dataset on every rank (fixed seeds); each rank takes a shard
    g = torch.Generator().manual_seed(1234)
    d_in = 32
    X = torch.randn(args.rows, d_in, generator=g)
    w_true = torch.randn(d_in, 1, generator=g)
    y = torch.tanh(X @ w_true) + 0.05 * torch.randn(args.rows, 1, generator=g)
    lo, hi = shard(args.rows, rank, world)
    xs, ys = X[lo:hi].to(dev), y[lo:hi].to(dev)
    torch.manual_seed(0)
    bias = bool(args.bias)
    layers = [torch.nn.Linear(d_in, args.hidden, bias=bias), torch.nn.Tanh()]
    for _ in range(args.layers - 1):
        layers += [torch.nn.Linear(args.hidden, args.hidden, bias=bias), torch.nn.Tanh()]
    model = torch.nn.Sequential(*layers, torch.nn.Linear(args.hidden, 1)).to(dev)
    if args.safe_linear:
        graph_safe_linear(model)
    buckets = GradientBuckets(model.parameters(), bucket_mb=args.bucket_mb)
    flat = {"p%d" % i: p.data for i, p in enumerate(model.parameters())}

    on_gpu = dev.type == "cuda"

    def save(next_step):
        if on_gpu:  # HBM snapshot + async pinned mirror; serialised only if a peer asks
            rabit.checkpoint_tensors(flat, meta={"next": next_step})
        else:
            rabit.checkpoint({"next": next_step,
                              "params": {k: v.numpy().copy() for k, v in flat.items()}})

    if on_gpu:
        version, meta = rabit.load_checkpoint_tensors(flat)
    else:
        version, meta = rabit.load_checkpoint()
        if version > 0:
            for k, v in flat.items():
                v.copy_(torch.from_numpy(meta["params"][k]))
    start = meta["next"] if version > 0 else 0
    if version > 0:
        print("[%d] resumed at version %d, step %d" % (rank, version, start), flush=True)
    def compute():
        loss = torch.nn.functional.mse_loss(model(xs), ys)
        buckets.backward(loss)  # gradients straight into the HBM buckets (graph-safe)
        return loss

    step_fn = GraphedStep(compute) if (args.graph and dev.type == "cuda") else compute
    for step in range(start, args.steps):
        loss = step_fn()
        if args.trace_steps:
            local = [hashlib.sha1(b.detach().cpu().numpy().tobytes()).hexdigest()[:8]
                     for b in buckets.buckets]
        buckets.reduce()
        if args.trace_steps:
            red = [hashlib.sha1(b.detach().cpu().numpy().tobytes()).hexdigest()[:8]
                   for b in buckets.buckets]
            wts = hashlib.sha1(b"".join(p.detach().cpu().numpy().tobytes()
                                        for p in model.parameters())).hexdigest()[:8]
            print("[%d] TRACE step %d weights %s local %s reduced %s" % (
                rank, step, wts, ",".join(local), ",".join(red)), flush=True)  # average over ranks; replayed from the survivors' logs after a restart
        with torch.no_grad():
            for p in model.parameters():
                p.add_(p.grad, alpha=-args.lr)
        if (step + 1) % args.ckpt == 0:
            save(step + 1)
        if rank == 0:
            print("[0] step %d local loss %.6f" % (step, loss.item()), flush=True)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    digest = hashlib.sha1(b"".join(p.detach().cpu().numpy().tobytes()
                                   for p in model.parameters())).hexdigest()[:16]
    # every rank must hold the same weights
    h = int(digest, 16) & ((1 << 62) - 1)
    lo_h = rabit.allreduce(np.array([h], dtype=np.int64), rabit.MIN)[0]
    hi_h = rabit.allreduce(np.array([h], dtype=np.int64), rabit.MAX)[0]
    assert lo_h == hi_h, "ranks disagree on the weights"
    st = rabit.stats()
    rabit.finalize()
    print("[%d] DPTRAIN OK weights=%s device_ops=%d replays=%d graphed=%d" % (
        rank, digest, st["n_device_ops"], st["n_device_replays"],
        int(getattr(step_fn, "captured", False))), flush=True)


if __name__ == "__main__":
    main()
