"""Time rabit.checkpoint_tensors of a 256 MiB HBM model at world 1 (BASELINE config 5's
checkpoint cost): median wall time of the call, and of the call plus a wait for the caller's
stream (the snapshot), over reps with a settle gap so the previous host mirror has finished."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
import rabit_amd as rabit  # noqa: E402
from rabit_amd.tracker import RabitTracker  # noqa: E402

tr = RabitTracker("127.0.0.1", 1, port=9391, port_end=9491, print_fn=lambda m: None).start(1)
rabit.init(rabit_tracker_uri="127.0.0.1", rabit_tracker_port=tr.port, rabit_task_id=0,
           rabit_world_size=1, rabit_world1_fastpath=0, rabit_device=0)
model = torch.rand((256 << 20) // 4, device="cuda")
rabit.checkpoint_tensors({"w": model}, meta={"it": 0})
call, total = [], []
for i in range(int(sys.argv[1]) if len(sys.argv) > 1 else 8):
    time.sleep(0.05)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    rabit.checkpoint_tensors({"w": model}, meta={"it": i + 1})
    t1 = time.perf_counter()
    torch.cuda.current_stream().synchronize()
    t2 = time.perf_counter()
    call.append(t1 - t0)
    total.append(t2 - t0)
print("checkpoint_256MiB call_us=%.1f total_us=%.1f" % (np.median(call) * 1e6,
                                                         np.median(total) * 1e6), flush=True)
rabit.finalize()
tr.join(10)
