"""A recovery epoch adopts the survivors' calibration instead of re-measuring (ranks share GPU 0;
rabit_device_calibrate_test=1 runs the calibration without RCCL).  Rank 1 is killed after the
first checkpoint; when the transports come back up every rank (the restarted one included)
takes the lowest surviving rank's routing, verified by one op per transport, and no rank
calibrates again.  Each iteration: device allreduces at three sizes, checked, then a checkpoint.
The recovery phase breakdown (stats()["recovery_phases_s"]) is printed for the profile."""
import json
import sys

import torch

import rabit_amd as rabit

rabit.init(sys.argv[1:], lib="mock", rabit_device=0, rabit_device_calibrate_test=1,
           rabit_device_peer_timeout_sec=20)
rank, world = rabit.get_rank(), rabit.get_world_size()
dev = torch.device("cuda", 0)
w = torch.zeros(4, device=dev)
version, meta = rabit.load_checkpoint_tensors({"w": w})
for it in range(version, 3):
    for n in (1000, 300000, 3 << 20):
        x = torch.full((n,), float(rank + 1 + it), device=dev)
        rabit.allreduce(x, rabit.SUM)
        assert torch.all(x == world * (world + 1) / 2 + world * it), (it, n)
    w.add_(1.0)
    rabit.checkpoint_tensors({"w": w}, meta={"it": it + 1})
torch.cuda.synchronize()
assert torch.all(w == 3.0), w
st = rabit.stats()
ph = st["recovery_phases_s"]
restarted = version > 0
rabit.finalize()
print("[%d] ADOPT %s" % (rank, json.dumps({"restarted": restarted, "phases": ph,
                                           "bands": st["calib_matrix"].get("form_bands")})),
      flush=True)
if "mock=1,1,0,0" in sys.argv[1:]:
    # every rank calibrated once at most (the first epoch), and the recovery epoch adopted
    assert ph["calibrations"] == (0 if restarted else 1), ph
    assert ph["adoptions"] >= 1, ph
print("[%d] CALIBADOPT OK" % rank, flush=True)
