"""Model families built on the rabit engine (data-parallel, fault tolerant):

KMeans      per-cluster statistics through a lazy-prepare allreduce
LinearModel logistic / least-squares regression, L-BFGS on allreduced [loss | grad]
HistGBDT    histogram gradient boosting: (node, feature, bin) histograms allreduced per level

All accept a local row shard as a torch tensor on CPU (TCP plane) or HBM (RCCL plane).
"""
from .gbdt import HistGBDT  # noqa: F401
from .kmeans import KMeans  # noqa: F401
from .linear import LinearModel  # noqa: F401
