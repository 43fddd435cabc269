"""rabit_amd.utils: per-rank Chrome traces from a 3-worker job merged and summarised."""
import glob
import json
import os
import sys

from rabit_amd.launcher import LocalJob
from rabit_amd.utils import Timer, merge_traces, params_to_args, summarize_trace

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_timer_and_params():
    t = Timer()
    for _ in range(3):
        with t:
            pass
    assert t.count == 3 and t.mean >= 0.0
    assert params_to_args(rabit_debug=1, rabit_timeout=0) == ["rabit_debug=1", "rabit_timeout=0"]


def test_merge_traces(tmp_path, native_build):
    script = os.path.join(ROOT, "tests", "scripts", "trace_dump.py")
    job = LocalJob([sys.executable, script, str(tmp_path)], 3, 1, capture=True, timeout=120,
                   print_fn=lambda m: None, tracker_port=9391)
    rc = job.run()
    out = "".join("".join(o) for o in job.outputs)
    assert rc == 0, out[-3000:]
    paths = sorted(glob.glob(str(tmp_path / "trace_*.json")))
    assert len(paths) == 3
    merged = str(tmp_path / "merged.json")
    n = merge_traces(paths, merged)
    with open(merged) as f:
        data = json.load(f)
    assert len(data["traceEvents"]) == n and n >= 3 * 7
    assert {e["pid"] for e in data["traceEvents"]} == {0, 1, 2}
    summary = summarize_trace(merged)
    assert summary["allreduce"]["count"] == 15
    assert summary["checkpoint"]["count"] == 3
