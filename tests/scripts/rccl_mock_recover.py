"""An RCCL enqueue error inside the robust engine is recovered, not fatal.

World 1 on one GPU with world-1 device ops routed through a one-rank RCCL communicator
(rabit_device_world1_transport=1, rabit_device_algo=rccl).  rabit_mock_rccl_error=N makes the
N-th RCCL enqueue return ncclRemoteError: the device plane aborts the communicator and returns
kAborted, CheckAndRecover re-links through the tracker, a new device epoch is built, and the
op is retried.  Prints one JSON line with the engine stats; exits non-zero on a wrong result."""
import json
import sys

import torch

import rabit_amd as rabit
from rabit_amd.tracker import RabitTracker

fail_at = int(sys.argv[1]) if len(sys.argv) > 1 else 3
tracker = RabitTracker("127.0.0.1", 1, port=9471, print_fn=lambda m: None).start(1)
rabit.init(lib="standard", rabit_tracker_uri="127.0.0.1", rabit_tracker_port=tracker.port,
           rabit_task_id=0, rabit_world_size=1, rabit_world1_fastpath=0,
           rabit_device_world1_transport=1, rabit_device_algo="rccl", rabit_device=0,
           rabit_mock_rccl_error=fail_at)
dev = torch.device("cuda", 0)
ok = True
for i in range(6):
    x = torch.arange(1 << 18, device=dev, dtype=torch.float32).remainder_(101) + i
    want = x.clone()
    rabit.allreduce(x, rabit.SUM)
    torch.cuda.synchronize()
    ok = ok and bool(torch.equal(x, want))
b = torch.arange(4096, device=dev, dtype=torch.int32)
rabit.broadcast_tensor(b, 0)
ok = ok and bool(torch.equal(b.cpu(), torch.arange(4096, dtype=torch.int32)))
st = rabit.stats()
print(json.dumps({"ok": ok, "rccl_aborts": st["rccl_aborts"], "rccl_calls": st["rccl_calls"],
                  "rccl_settled": st["rccl_settled"],
                  "n_recover_events": st["n_recover_events"], "device_epoch": st["device_epoch"],
                  "n_allreduce": st["n_allreduce"]}), flush=True)
rabit.finalize()
tracker.join(30)
sys.exit(0 if ok else 1)
