#!/usr/bin/env python3
"""Kernel-order evidence for the zero-copy registry ("a rocprofv3 trace shows
no stage CopyTileKernel before the first barrier").

Worker (one rank, started by tools/zero_copy_trace.sh under its own rocprofv3 --kernel-trace):
the base engine (no result-log copies, so every CopyTileKernel is a stage copy) allreduces one
128 MiB torch allocation OPS times with zero copy on, then OPS times with it off
(rabit.set_zero_copy(0)); every result is checked against the closed form.  Each op sits between
two host barriers (rabit.allreduce of a 1-int host array, no device kernel) and its wall time is
recorded.

Analysis (`--analyze <kernel_trace.csv> <worker log> [out.json]`): the rabit kernels of each op in
start order, the op's GPU span, and how many CopyTileKernel ran before its first
PeerBarrierKernel.
"""
import csv
import json
import os
import sys
import time

OPS = 10
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def worker():
    import numpy as np
    import torch
    import rabit_amd as rabit
    from rabit_amd.torchrun import init_from_env

    ctx = init_from_env(lib="base", rabit_world1_fastpath=0, rabit_device=0,
                        rabit_device_peer_buffer="32M")
    rank, world = rabit.get_rank(), rabit.get_world_size()
    dev = torch.device("cuda", 0)
    n = 32 << 20
    x = torch.empty(n, dtype=torch.float32, device=dev)
    base = torch.arange(n, device=dev, dtype=torch.float32).remainder(7)
    marks = []
    for zc in (1, 0):
        rabit.set_zero_copy(zc)
        for i in range(OPS):
            x.copy_(base + rank + i)
            torch.cuda.synchronize()
            rabit.allreduce(np.zeros(1, dtype=np.int32), rabit.SUM)
            t0 = time.time_ns()
            rabit.allreduce(x, rabit.SUM)
            torch.cuda.synchronize()
            t1 = time.time_ns()
            want = base * world + i * world + world * (world - 1) / 2
            assert torch.equal(x, want), (zc, i)
            marks.append({"zero_copy": zc, "op": i, "t0_ns": t0, "t1_ns": t1,
                          "us": (t1 - t0) / 1e3})
    st = rabit.stats()
    print("ZCTRACE " + json.dumps({"rank": rank, "world": world, "marks": marks,
                                   "registry": st.get("zero_copy_registry")}), flush=True)
    del x
    ctx.finalize()


def short_name(name):
    name = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return name.split("(")[0].split("<")[0].split("::")[-1]


def analyze(trace_csv, log):
    """each op of the worker is one run of consecutive rabit kernels between torch's own (the
    input fill before it, the check after it) that contains a barrier; the last 2 x OPS such runs
    are the timed ops, in order (zero copy on, then off)"""
    marks = None
    for line in open(log, encoding="utf-8", errors="replace"):
        if line.startswith("ZCTRACE "):
            marks = json.loads(line[len("ZCTRACE "):])
    if marks is None:
        raise SystemExit("no ZCTRACE line in " + log)
    rows = []
    with open(trace_csv, newline="") as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    runs, cur = [], []
    for s, e, name in rows:
        if "rabit::device" in name:
            cur.append((s, e, short_name(name)))
        elif cur:
            runs.append(cur)
            cur = []
    if cur:
        runs.append(cur)
    runs = [r for r in runs if any(k[2] == "PeerBarrierKernel" for k in r)]
    windows = marks["marks"]
    if len(runs) < len(windows):
        raise SystemExit("%d ops in the trace, %d timed" % (len(runs), len(windows)))
    runs = runs[-len(windows):]
    out = {"rank": marks["rank"], "world": marks["world"], "registry": marks["registry"],
           "ops": []}
    for w, run in zip(windows, runs):
        names = [k[2] for k in run]
        first_bar = names.index("PeerBarrierKernel")
        out["ops"].append({
            "zero_copy": w["zero_copy"], "op": w["op"], "wall_us": round(w["us"], 1),
            "gpu_span_us": round((run[-1][1] - run[0][0]) / 1e3, 1),
            "stage_copies_before_first_barrier": names[:first_bar].count("CopyTileKernel"),
            "kernels": names})
    for zc in (1, 0):
        ops = [o for o in out["ops"] if o["zero_copy"] == zc and o["op"] >= 2]
        spans = sorted(o["gpu_span_us"] for o in ops)
        out["zero_copy_on" if zc else "zero_copy_off"] = {
            "median_gpu_span_us_ops_2_on": spans[len(spans) // 2] if spans else None,
            "stage_copies_before_first_barrier_ops_2_on":
                [o["stage_copies_before_first_barrier"] for o in ops]}
    return out


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--analyze":
        res = analyze(sys.argv[2], sys.argv[3])
        dst = sys.argv[4] if len(sys.argv) > 4 else None
        text = json.dumps(res, indent=1)
        if dst:
            with open(dst, "w") as f:
                f.write(text + "\n")
        print(json.dumps({k: v for k, v in res.items() if k != "ops"}))
        for o in res["ops"]:
            if o["op"] in (0, 2):
                print("zero_copy=%d op %d: %.1f us: %s" % (o["zero_copy"], o["op"],
                                                          o["gpu_span_us"], " ".join(o["kernels"])))
    else:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        worker()
