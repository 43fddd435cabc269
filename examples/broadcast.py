"""Broadcast (semantics of the reference's guide/broadcast.py): rank 0 holds a Python object,
every worker ends with a copy.  Objects travel pickled over the host control plane; tensors in
HBM go through `rabit.broadcast_tensor`, which moves the bytes GPU to GPU.

    python -m rabit_amd.launcher -n 3 python examples/broadcast.py
"""
import rabit_amd as rabit


def main():
    rabit.init()
    rank = rabit.get_rank()
    obj = {"hello world": 100, 2: 3} if rank == 0 else None
    print('@node[%d] before-broadcast: s="%s"' % (rank, obj), flush=True)
    obj = rabit.broadcast(obj, 0)
    print('@node[%d] after-broadcast: s="%s"' % (rank, obj), flush=True)
    rabit.finalize()


if __name__ == "__main__":
    main()
