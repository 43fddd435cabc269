"""Lazy preparation (semantics of the reference's guide/lazy_allreduce.py): the buffer is filled
by a prepare callback that the engine calls right before the reduction and skips when the
result is replayed from a peer's result log after a failure.  Run it under the mock engine with
a kill (`lib=mock mock=0,0,0,0`) to see a restarted worker take the result without preparing.

On the GPU the common prepare functions do not need a Python callback at all:
`rabit.allreduce_prepared(out, grad, rabit.SUM, rabit.PREP_SQUARE)` squares the gradient inside
the reduction kernel (one pass over HBM, skipped on replay like the callback).

    python -m rabit_amd.launcher -n 2 python examples/lazy_allreduce.py
"""
import numpy as np

import rabit_amd as rabit


def main():
    rabit.init()
    rank = rabit.get_rank()
    buf = np.zeros(3)

    def fill(b):
        print("@node[%d] run prepare function" % rank, flush=True)
        b[:] = rank + np.arange(b.size)

    print("@node[%d] before-allreduce: a=%s" % (rank, buf), flush=True)
    buf = rabit.allreduce(buf, rabit.MAX, prepare_fun=fill)
    print("@node[%d] after-allreduce-max: a=%s" % (rank, buf), flush=True)
    buf = rabit.allreduce(buf, rabit.SUM)
    print("@node[%d] after-allreduce-sum: a=%s" % (rank, buf), flush=True)
    rabit.finalize()


if __name__ == "__main__":
    main()
