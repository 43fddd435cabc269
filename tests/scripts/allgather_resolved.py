"""Device Allgather over the direct transport with the slice layout resolved on the device
(no host round per op; rabit_device_allgather_resolve=0 restores the host round for the
comparison).  Variable, wrapping slices; the same layout repeated, then changed; windows larger
than the stage buffer (several barriers per op); int8 payloads checked byte for byte.  Rank 0
prints the median latency of a 1 MiB allgather (4 slices)."""
import sys
import time

import numpy as np
import torch

import rabit_amd as rabit

rabit.init(sys.argv[1:], lib="standard", rabit_device=0, rabit_device_peer_buffer="1M",
           rabit_device_peer_timeout_sec=20)
rank, world = rabit.get_rank(), rabit.get_world_size()
dev = torch.device("cuda", 0)


def layout(total, seed):
    """slice sizes that sum to total (some empty), starting at a rotating offset (wraps)"""
    rng = np.random.RandomState(seed)
    cuts = np.sort(rng.randint(0, total + 1, size=world - 1))
    sizes = np.diff(np.concatenate([[0], cuts, [total]])).astype(np.int64)
    start = int(rng.randint(0, total))
    begins = (start + np.concatenate([[0], np.cumsum(sizes)[:-1]])) % total
    return begins, sizes


ops = 0
for total, seeds in ((1000, (1, 1, 1, 2)), (3 << 19, (3, 3, 4)), ((7 << 19) + 13, (5, 6, 6))):
    for seed in seeds:
        begins, sizes = layout(total, seed)
        want = ((torch.arange(total, dtype=torch.int64) * 131 + seed) % 251).to(torch.uint8)
        buf = torch.zeros(total, dtype=torch.uint8, device=dev)
        b, z = int(begins[rank]), int(sizes[rank])
        idx = (torch.arange(z, dtype=torch.int64) + b) % total
        buf[idx.to(dev)] = want[idx].to(dev)
        rabit.allgather_slice(buf, b, z, int(sizes[(rank - 1) % world]))
        assert torch.equal(buf.cpu(), want), (total, seed)
        ops += 1
# latency of a 1 MiB allgather with equal slices
total = 1 << 20
buf = torch.zeros(total, dtype=torch.uint8, device=dev)
per = total // world
ts = []
for i in range(30):
    torch.cuda.synchronize()
    rabit.allreduce(np.zeros(1, dtype=np.int32), rabit.SUM)
    t0 = time.perf_counter()
    rabit.allgather_slice(buf, rank * per, per if rank < world - 1 else total - rank * per,
                          per if rank > 0 else total - (world - 1) * per)
    torch.cuda.synchronize()
    ts.append(time.perf_counter() - t0)
    if i % 10 == 9:
        rabit.checkpoint(None)
med = float(rabit.allreduce(np.array([float(np.median(ts[5:]))]), rabit.MAX)[0])
st = rabit.stats()
resolve = "rabit_device_allgather_resolve=0" not in sys.argv[1:]
assert (st["resolved_allgathers"] > 0) == resolve, st["resolved_allgathers"]
rabit.finalize()
print("[%d] AGRESOLVED OK ops=%d resolved=%d allgather_1MiB_us=%.1f"
      % (rank, ops, st["resolved_allgathers"], med * 1e6), flush=True)
