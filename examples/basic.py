"""What Allreduce does (semantics of the reference's guide/basic.py): every worker holds
a[i] = rank + i, and the workers agree first on the element-wise Max, then on the Sum.

The same two reductions run on a host numpy array and, when the worker has a GPU, on an HBM
tensor (the device plane: RCCL or the direct xGMI transport between GPUs); both must agree.

    python -m rabit_amd.launcher -n 4 python examples/basic.py
"""
import numpy as np

import rabit_amd as rabit


def hbm_copy(values):
    """the same values as a torch tensor in HBM, or None on a CPU-only worker"""
    try:
        import torch
    except ImportError:
        return None
    if not torch.cuda.is_available():
        return None
    return torch.as_tensor(values, device="cuda")


def show(tag, values):
    print("@node[%d] %s: a=%s" % (rabit.get_rank(), tag, values), flush=True)


def main():
    rabit.init()
    host = np.arange(3, dtype=np.float64) + rabit.get_rank()
    dev = hbm_copy(host)
    show("before-allreduce", host)
    for tag, op in (("after-allreduce-max", rabit.MAX), ("after-allreduce-sum", rabit.SUM)):
        host = rabit.allreduce(host, op)
        if dev is not None:
            rabit.allreduce(dev, op)
            assert np.array_equal(dev.cpu().numpy(), host), (tag, dev, host)
        show(tag, host)
    rabit.finalize()


if __name__ == "__main__":
    main()
