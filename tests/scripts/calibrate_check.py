"""Calibration control flow on a shared GPU (rabit_device_calibrate_test=1: the RCCL leg runs
on the direct transport too).  Checks that every rank reports the same decision and that
collectives of both sides of the threshold give correct results afterwards."""
import sys

import numpy as np
import torch

import rabit_amd as rabit

rabit.init(sys.argv[1:], lib="standard", rabit_device=0, rabit_device_calibrate_test=1)
rank, world = rabit.get_rank(), rabit.get_world_size()
dev = torch.device("cuda", 0)
for n in (1000, 3 << 20):
    x = torch.full((n,), float(rank + 1), device=dev)
    rabit.allreduce(x, rabit.SUM)
    assert torch.all(x == world * (world + 1) / 2), n
st = rabit.stats()
calib = st["calib_us"]
assert all(c > 0 for c in calib), calib
thr = st["device_direct_min"]
lo = rabit.allreduce(np.array([thr]), rabit.MIN)[0]
hi = rabit.allreduce(np.array([thr]), rabit.MAX)[0]
assert lo == hi, (lo, hi)
# the small-op window (direct below a crossover when RCCL wins at the large point) is uniform too,
# and never overlaps the large-op threshold
below = st["device_direct_below"]
blo = rabit.allreduce(np.array([below]), rabit.MIN)[0]
bhi = rabit.allreduce(np.array([below]), rabit.MAX)[0]
assert blo == bhi, (blo, bhi)
assert below == 0 or thr >= 2 ** 63, (below, thr)
# the push variant was timed and the pull/push choice is the same everywhere
assert st["calib_push_us"] > 0, st
push = rabit.allreduce(np.array([st["direct_push"]]), rabit.SUM)[0]
assert push in (0, world), push
# the forms of the two-shot path were timed and verified (pull/push x classic and the pipelined
# push form; the fused forms too with rabit_device_fused=auto), and the chosen form is the same
# everywhere
forms = st["calib_forms_us"]
fused_auto = "rabit_device_fused=auto" in sys.argv[1:]
assert len(forms) == 5 and forms[0] > 0 and forms[2] > 0 and forms[4] > 0, forms
pipe = rabit.allreduce(np.array([st["direct_pipeline"]]), rabit.SUM)[0]
assert pipe in (0, world), pipe
if fused_auto:
    assert all(f > 0 for f in forms[:4]), forms
else:
    assert forms[1] == -1 and forms[3] == -1 and st["direct_fused"] == 0, (forms, st)
fused = rabit.allreduce(np.array([st["direct_fused"]]), rabit.SUM)[0]
assert fused in (0, world), fused
# the piecewise calibration: every candidate at 5 sizes (64 KiB .. 128 MiB), size bands for the
# transport and the direct form, the same on every rank; every measured point routes to its own
# fastest form
cm = st["calib_matrix"]
assert cm["bytes"] == [64 << 10, 1 << 20, 4 << 20, 32 << 20, 128 << 20], cm
assert len(cm["us"]["rccl"]) == 5 and all(v > 0 for v in cm["us"]["pull-classic"]), cm
assert cm["transport_bands"] and cm["form_bands"] and cm["form_bands"][0]["from"] == 0, cm
import json, zlib  # noqa: E401
h = zlib.crc32(json.dumps(cm["form_bands"], sort_keys=True).encode()) & 0x7fffffff
assert rabit.allreduce(np.array([h]), rabit.MIN)[0] == rabit.allreduce(np.array([h]), rabit.MAX)[0]
# the fused forms are timed but never routed to while ranks share a GPU (their tile hand-offs
# need every rank's grid resident at once, which separate processes on one GPU do not get)
unrouted = set(cm["unrouted_forms"])
assert unrouted == ({"pull-fused", "push-fused"} if fused_auto else set()), unrouted
for i, nb in enumerate(cm["bytes"]):
    band = [b for b in cm["form_bands"] if b["from"] <= nb][-1]["form"]
    times = {k: v[i] for k, v in cm["us"].items() if k != "rccl" and k not in unrouted and v[i] > 0}
    assert band == min(times, key=times.get), (nb, band, times)
ph = st["recovery_phases_s"]
assert ph["bringups"] == 1 and ph["calibrations"] == 1 and ph["adoptions"] == 0, ph
# with a symmetric heap that has room, the calibration reads its inputs from the heap's tail
want_heap = any(a.startswith("rabit_device_symmetric_heap=") for a in sys.argv[1:])
assert st["calib_heap_src"] == (1 if want_heap else 0), st
# the broadcast calibration ran after the allreduce one (both legs timed and the direct result
# verified), its routing is the same everywhere, and broadcasts on both sides of it are correct
bc = st["calib_bcast_us"]
assert len(bc) == 4 and all(c > 0 for c in bc), bc
assert st["bcast_routed"] == 1, st
for key in ("bcast_direct_min", "bcast_direct_below"):
    v = st[key]
    assert rabit.allreduce(np.array([v]), rabit.MIN)[0] == rabit.allreduce(np.array([v]), rabit.MAX)[0], key
for nbytes in (333, (5 << 20) + 1):
    want = torch.arange(nbytes, dtype=torch.int64).remainder(241).to(torch.uint8)
    b = want.to(dev) if rank == world - 1 else torch.zeros(nbytes, dtype=torch.uint8, device=dev)
    rabit.broadcast_tensor(b, world - 1)
    assert torch.equal(b.cpu(), want), nbytes
rabit.finalize()
print("[%d] CALIB OK thr=%s calib=%s" % (rank, thr, calib), flush=True)
