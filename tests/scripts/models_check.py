"""Train the model families on a row-sharded synthetic dataset and verify on every rank."""
import hashlib
import sys

import numpy as np
import torch

import rabit_amd as rabit
from rabit_amd.models import HistGBDT, KMeans, LinearModel
from rabit_amd.parallel.data_parallel import shard

which = sys.argv[1]
rabit.init(sys.argv[2:], lib="mock")
rank, world = rabit.get_rank(), rabit.get_world_size()
dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")


def same_everywhere(arr):
    h = int(hashlib.sha1(np.ascontiguousarray(arr).tobytes()).hexdigest()[:12], 16)
    lo = rabit.allreduce(np.array([h], dtype=np.int64), rabit.MIN)[0]
    hi = rabit.allreduce(np.array([h], dtype=np.int64), rabit.MAX)[0]
    return lo == hi


g = torch.Generator().manual_seed(7)
if which == "kmeans":
    centers = torch.tensor([[0.0, 0.0], [10.0, 10.0], [-10.0, 10.0]], dtype=torch.float64)
    n = 3000
    lab = torch.randint(0, 3, (n,), generator=g)
    X = centers[lab] + 0.5 * torch.randn(n, 2, generator=g, dtype=torch.float64)
    b, e = shard(n, rank, world)
    km = KMeans(3, n_iter=8, seed=1)
    c = km.fit(X[b:e].to(dev)).cpu()
    # every true center has a centroid nearby
    d = torch.cdist(centers, c).min(dim=1).values
    assert float(d.max()) < 0.2, (c, d)
    assert same_everywhere(c.numpy())
elif which == "linear":
    n, dfeat = 4000, 8
    X = torch.randn(n, dfeat, generator=g, dtype=torch.float64)
    w_true = torch.arange(1, dfeat + 1, dtype=torch.float64) / dfeat
    y = torch.sign(X @ w_true + 0.1 * torch.randn(n, generator=g, dtype=torch.float64))
    b, e = shard(n, rank, world)
    lm = LinearModel(dfeat, "logistic", n_iter=15, device=dev)
    w = lm.fit(X[b:e], y[b:e]).cpu()
    acc = float((lm.predict(X).cpu() == y).double().mean())
    assert acc > 0.95, acc
    assert same_everywhere(w.numpy().round(10))
    print("[%d] final loss %.8f" % (rank, lm.history[-1]), flush=True)
elif which == "gbdt":
    n, dfeat = 3000, 5
    X = torch.rand(n, dfeat, generator=g, dtype=torch.float64)
    y = ((X[:, 0] > 0.5) ^ (X[:, 1] > 0.3)).double()
    b, e = shard(n, rank, world)
    gb = HistGBDT(n_trees=6, max_depth=3, n_bins=32)
    gb.fit(X[b:e].to(dev), y[b:e].to(dev))
    p = gb.predict_proba(X.to(dev)).cpu()
    acc = float(((p > 0.5).double() == y).double().mean())
    assert acc > 0.95, acc
    feats = np.concatenate([t["feature"].numpy() for t in gb.trees])
    assert same_everywhere(feats)
    assert gb.hist_allreduce_bytes > 0
rabit.finalize()
print("[%d] MODEL OK" % rank, flush=True)
