"""dp_train.py digests: eager clean, graphed clean, graphed with failures (3 ranks)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)
from test_examples import run_dp_train  # noqa: E402

args = ["--hidden", "256", "--layers", "6", "--bucket-mb", "1"] + sys.argv[1:]
CASES = [("eager", [], 1), ("graph", ["--graph", "1"], 1),
         ("graph_fail", ["--graph", "1", "mock=1,2,1,0", "mock=2,3,0,0"], 3),
         ("eager_fail", ["mock=1,2,1,0", "mock=2,3,0,0"], 3),
         ("graph_fail_r1", ["--graph", "1", "mock=1,2,1,0"], 3),
         ("graph_fail_r2", ["--graph", "1", "mock=2,3,0,0"], 3),
         ("graph_fail_r0_v1", ["--graph", "1", "mock=0,1,0,0"], 3),
         ("graph_fail_r1_v3", ["--graph", "1", "mock=1,3,1,0"], 3)]
for name, extra, att in CASES:
    d, job, out = run_dp_train(3, att, args + extra)
    print(name, d, job.attempts, flush=True)
