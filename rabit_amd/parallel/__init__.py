"""Data-parallel building blocks on top of the rabit engine (rabit is the DP substrate:
SURVEY §2.9 — every worker holds a shard and Allreduce aggregates statistics).

GradientBuckets   flat HBM gradient buckets (gradients are views into them, so backward
                  writes straight into the buffers that are reduced: zero packing copies),
                  one large fault-tolerant allreduce per bucket, averaging fused into the
                  lazy-prepare kernel.
FaultTolerantLoop resume-from-checkpoint training loop (LoadCheckPoint / CheckPoint every
                  k steps), the rabit programming model for iterative jobs.
GraphedStep       replays the launch-bound device part of an iteration (forward, backward,
                  bucket zeroing) as one hipGraph; the collectives stay outside it.
CommThread,       the engine on its own host thread; bucket allreduces start from backward
OverlappedBuckets hooks and run on their own HIP stream while backward continues.
"""
from .data_parallel import FaultTolerantLoop, GradientBuckets  # noqa: F401
from .graphs import GraphedStep, graph_safe_linear  # noqa: F401
from .overlap import CommThread, OverlappedBuckets  # noqa: F401
