#!/usr/bin/env python3
"""Head-to-head of the reference's own speed benchmark against xrabit on the same machine.

The reference (bobjiang82/rabit) publishes no numbers, so this measures them:
`tools/refbuild/build_reference.sh` compiles the reference's sources and its
`test/speed_test.cc` (BASELINE.json's headline benchmark) into build/ref, and this script runs
that program and xrabit's `tests/cpp/speed_test.cc` (same arguments, same output lines) under
the same launcher and tracker (xrabit's tracker speaks the reference's wire protocol, SURVEY
Appendix A) for each world size, then prints one JSON line per (implementation, world).

    python tools/refbuild/compare_speed.py --worlds 1 2 4 8 --n 33554432 --nrep 3

Implementations:
  reference  - the reference robust engine, host buffers over TCP (its only data path)
  xrabit     - xrabit's robust engine, host buffers (shared memory between co-located ranks
               for large ops, TCP otherwise)
  xrabit_tcp - xrabit's host path over loopback TCP only (rabit_host_shm=0)
  xrabit_inplace - xrabit's robust engine copying the input into the result log first
               (rabit_host_out_of_place=0, the reference's scheme) for A/B runs
  xrabit_via_dev - host buffers staged through HBM onto the device transports
               (rabit_host_via_device=1; the MPI-engine role on a GPU node); large ops
               pipelined or whole as the timed choice finds faster (rabit_host_stage=auto)
  xrabit_via_dev_whole - the same with one whole pageable copy each way (rabit_host_stage=0),
               the round-1/2 form, for A/B runs
  xrabit_via_dev_pipe - always pipelined (rabit_host_stage=1)
  xrabit_dev - xrabit with HBM buffers (device=1); only at world 1 unless --dev-worlds is
               given (several ranks on one GPU share its HBM: not an xGMI number)
"""
import argparse
import json
import os
import re
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
LINE = re.compile(r"^(max|sum|bcast|tot)_tdiff(-speed)?: (?:mean=([0-9.eE+-]+), std=([0-9.eE+-]+) sec|"
                  r"([0-9.eE+-]+) MB/sec)")


def run(cmd, world, timeout, port):
    launcher = [sys.executable, "-m", "rabit_amd.launcher", "-n", str(world), "--port", str(port),
                "--timeout", str(timeout)]
    t0 = time.time()
    p = subprocess.run(launcher + ["--"] + cmd, cwd=ROOT, capture_output=True, text=True,
                       timeout=timeout + 30)
    wall = time.time() - t0
    res = {"rc": p.returncode, "wall_s": round(wall, 2)}
    for line in (p.stdout + p.stderr).splitlines():
        m = LINE.match(line.strip())
        if not m:
            continue
        kind, speed, mean, std, mbs = m.groups()
        if speed:
            res[kind + "_MBps"] = float(mbs)
        else:
            res[kind + "_mean_s"] = float(mean)
            res[kind + "_std_s"] = float(std)
    if p.returncode != 0:
        res["tail"] = (p.stdout + p.stderr)[-1500:]
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", type=int, nargs="+", default=[1, 2, 4])
    ap.add_argument("--dev-worlds", type=int, nargs="*", default=[1])
    ap.add_argument("--n", type=int, default=33554432, help="float32 elements (128 MiB)")
    ap.add_argument("--nrep", type=int, default=3)
    ap.add_argument("--timeout", type=float, default=600)
    ap.add_argument("--impl", nargs="+", default=["reference", "xrabit", "xrabit_dev"])
    ap.add_argument("--out", default=None, help="also append the JSON lines to this file")
    args = ap.parse_args()
    ref = os.path.join(ROOT, "build", "ref", "speed_test")
    ours = os.path.join(ROOT, "build", "bin", "speed_test")
    if "reference" in args.impl and not os.path.exists(ref):
        subprocess.check_call(["bash", os.path.join(ROOT, "tools", "refbuild",
                                                    "build_reference.sh")])
    port = 9300
    for world in args.worlds:
        for impl in args.impl:
            if impl == "xrabit_dev" and world not in args.dev_worlds:
                continue
            cmd = {"reference": [ref, str(args.n), str(args.nrep)],
                   "xrabit": [ours, str(args.n), str(args.nrep)],
                   "xrabit_tcp": [ours, str(args.n), str(args.nrep), "rabit_host_shm=0"],
                   "xrabit_inplace": [ours, str(args.n), str(args.nrep),
                                      "rabit_host_out_of_place=0"],
                   "xrabit_via_dev": [ours, str(args.n), str(args.nrep),
                                      "rabit_host_via_device=1"],
                   "xrabit_via_dev_whole": [ours, str(args.n), str(args.nrep),
                                            "rabit_host_via_device=1", "rabit_host_stage=0"],
                   "xrabit_via_dev_pipe": [ours, str(args.n), str(args.nrep),
                                           "rabit_host_via_device=1", "rabit_host_stage=1"],
                   "xrabit_dev": [ours, str(args.n), str(args.nrep), "device=1",
                                  "rabit_world1_fastpath=0"]}[impl]
            port += 7
            rec = {"impl": impl, "world": world, "n": args.n, "nrep": args.nrep,
                   "bytes": args.n * 4}
            rec.update(run(cmd, world, args.timeout, port))
            line = json.dumps(rec)
            print(line, flush=True)
            if args.out:
                with open(args.out, "a") as f:
                    f.write(line + "\n")


if __name__ == "__main__":
    main()
