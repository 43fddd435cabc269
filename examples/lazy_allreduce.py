"""guide/lazy_allreduce.py equivalent: the prepare function fills the buffer right before the
reduction and is skipped when the result is recovered from peers after a failure."""
import numpy as np
import rabit_amd as rabit

rabit.init()
n = 3
rank = rabit.get_rank()
a = np.zeros(n)


def prepare(a):
    print('@node[%d] run prepare function' % rank)
    for i in range(n):
        a[i] = rank + i


print('@node[%d] before-allreduce: a=%s' % (rank, str(a)))
a = rabit.allreduce(a, rabit.MAX, prepare_fun=prepare)
print('@node[%d] after-allreduce-max: a=%s' % (rank, str(a)))
a = rabit.allreduce(a, rabit.SUM)
print('@node[%d] after-allreduce-sum: a=%s' % (rank, str(a)))
rabit.finalize()
