"""Free HBM of GPU 0 and the processes that hold the GPU (diagnosis of a slow headline)."""
import os
import subprocess
import sys

import torch

free, total = torch.cuda.mem_get_info(0)
print("%s free_hbm_GiB=%.1f total_GiB=%.1f" % (sys.argv[1] if len(sys.argv) > 1 else "",
                                              free / 2 ** 30, total / 2 ** 30), flush=True)
out = subprocess.run(["ps", "-eo", "pid,ppid,stat,etime,rss,args"], capture_output=True,
                     text=True).stdout
for line in out.splitlines():
    if "python" in line and "hbm_probe" not in line:
        print("  " + line[:200], flush=True)
# shared-memory segments (a killed worker leaves its own behind) and host memory
try:
    segs = [(f, os.path.getsize(os.path.join("/dev/shm", f))) for f in os.listdir("/dev/shm")]
    print("  /dev/shm: %d segments, %.1f MiB (xrabit: %d)" % (
        len(segs), sum(s for _, s in segs) / 2 ** 20,
        sum(1 for f, _ in segs if "xrabit" in f or "rabit" in f)), flush=True)
    print("  " + " ".join(l.split(":")[0] + "=" + l.split()[1] for l in open("/proc/meminfo")
                          if l.startswith(("MemAvailable", "Shmem:", "MemFree"))), flush=True)
except OSError as e:
    print("  /dev/shm: %s" % e, flush=True)
