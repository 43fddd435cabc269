"""Per-step gradient digests of dp_train.py, graphed, clean vs one killed worker."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)
from test_examples import run_dp_train  # noqa: E402

args = ["--hidden", "256", "--layers", "6", "--bucket-mb", "1", "--trace-steps", "1"]
for name, extra, att in [("graph", ["--graph", "1"], 1), ("eager", [], 1),
                         ("graph_fail_r1", ["--graph", "1", "mock=1,2,1,0"], 3)]:
    d, job, out = run_dp_train(3, att, args + extra)
    print("=====", name, d, job.attempts, flush=True)
    for line in out.splitlines():
        if "TRACE" in line or "resumed" in line or "Mock" in line:
            print(line, flush=True)
