"""Sweep driver for build/bin/speed_test (the reference's test/speed_runner.py: message sizes
x repeat counts x worker counts), on the local launcher instead of host files.

    python tools/speed_runner.py                      # host (TCP) plane, 2 and 4 workers
    python tools/speed_runner.py --device --workers 2 # HBM buffers (ranks share GPU 0 on a
                                                      # one-GPU box: direct IPC transport)

Prints one JSON line per (workers, n) with the per-op mean times and MB/s lines speed_test
reports through the tracker.
"""
import argparse
import json
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# the reference's sweep: n in {1e4, 1e5, 1e6, 1e7} with repeats {1e4, 1e3, 1e2, 10}
SWEEP = [(10000, 1000), (100000, 100), (1000000, 20), (10000000, 5)]


def run(workers, n, nrep, device, extra):
    prog = os.path.join(ROOT, "build", "bin", "speed_test")
    cmd = [sys.executable, "-m", "rabit_amd.launcher", "-n", str(workers), prog, str(n),
           str(nrep)] + (["device=1", "rabit_device=0"] if device else []) + list(extra)
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=900, cwd=ROOT)
    out = p.stdout + p.stderr
    rec = {"workers": workers, "n": n, "nrep": nrep, "device": device, "rc": p.returncode}
    for name in ("max_tdiff", "sum_tdiff", "bcast_tdiff", "tot_tdiff"):
        m = re.search(r"%s: mean=([0-9.eE+-]+)" % name, out)
        if m:
            rec[name + "_s"] = float(m.group(1))
        m = re.search(r"%s-speed: ([0-9.eE+-]+) MB/sec \(algbw ([0-9.]+) GB/s, busbw ([0-9.]+)"
                      % name, out)
        if m:
            rec[name + "_MBps"] = float(m.group(1))
            rec[name + "_busbw_GBps"] = float(m.group(3))
    if p.returncode != 0:
        rec["tail"] = out[-1000:]
    return rec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workers", type=int, nargs="+", default=[2, 4])
    ap.add_argument("--device", action="store_true")
    ap.add_argument("extra", nargs="*", help="rabit params passed to every worker")
    args = ap.parse_args()
    subprocess.check_call(["make", "-j8", "tests"], cwd=ROOT, stdout=subprocess.DEVNULL)
    for w in args.workers:
        for n, nrep in SWEEP:
            print(json.dumps(run(w, n, nrep, args.device, args.extra)), flush=True)


if __name__ == "__main__":
    main()
