"""Zero-copy allreduce from the symmetric heap over the direct transport (ranks share GPU 0).
Even ranks allocate their input in the heap (read in place by the peers), odd ranks use plain
torch memory (staged) — the mailbox protocol lets every rank choose for itself.  Several
sizes, a chunked one included, dtypes and ops; closed-form checks."""
import sys

import torch

import rabit_amd as rabit

rabit.init(sys.argv[1:], lib="standard", rabit_device=0, rabit_device_symmetric_heap="64M",
           rabit_device_peer_buffer="4M", rabit_device_peer_timeout_sec=20)
rank, world = rabit.get_rank(), rabit.get_world_size()
dev = torch.device("cuda", 0)
sym = rank % 2 == 0
cases = 0
for dtype in (torch.float32, torch.int32, torch.float64):
    for n in (1000, 1 << 20, (6 << 20) // torch.empty((), dtype=dtype).element_size() + 7):
        if sym:
            x = rabit.symmetric_empty(n, dtype)  # bump-allocated: reuse it for both ops
        else:
            x = torch.empty(n, dtype=dtype, device=dev)
        for op in (rabit.SUM, rabit.MAX):
            base = torch.arange(n, device=dev, dtype=torch.float64).remainder(7)
            x.copy_((base + rank).to(dtype))
            rabit.allreduce(x, op)
            if op == rabit.SUM:
                want = base * world + world * (world - 1) / 2
            else:
                want = base + (world - 1)
            assert torch.equal(x.double(), want), (dtype, n, op)
            cases += 1
st = rabit.stats()
if sym and world > 1:
    assert st["zero_copy_chunks"] > 0, st
rabit.finalize()
print("[%d] SYMMETRIC OK %d cases, zero-copy chunks %d" % (rank, cases, st["zero_copy_chunks"]),
      flush=True)
