"""bench.py's run-time guards (CPU): the deadline watcher names the phase and exits non-zero
before the headline exists; once the headline is measured, a stuck side measurement still ends
the run with exactly one JSON line on rank 0 (flagged) and exit status 0."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(body, timeout=60):
    code = "import sys, time; sys.path.insert(0, %r); import bench\n%s" % (ROOT, body)
    return subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                          timeout=timeout)


def test_deadline_before_headline_fails():
    p = _run("bench.phase('timed')\nbench.start_deadline(1, 0, 100)\ntime.sleep(30)")
    assert p.returncode == 3
    assert "phase 'timed'" in p.stderr
    assert p.stdout.strip() == ""


def test_stuck_side_measurement_still_prints_headline():
    p = _run("bench.start_deadline(100, 0, 1)\n"
             "bench.HEADLINE.update(rec={'metric': 'm', 'value': 1.0}, t=time.time())\n"
             "bench.phase('variant direct-push-fused/torch')\ntime.sleep(30)")
    assert p.returncode == 0, p.stderr
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    rec = json.loads(lines[0])
    assert rec["value"] == 1.0
    assert "direct-push-fused" in rec["post_headline_failure"]


def test_headline_printed_once_and_only_on_rank0():
    p = _run("bench.start_deadline(100, 0, 2)\n"
             "bench.HEADLINE.update(rec={'metric': 'm', 'value': 2.0}, t=time.time())\n"
             "bench.emit_headline()\nbench.phase('finalize')\ntime.sleep(30)")
    assert p.returncode == 0
    assert len([ln for ln in p.stdout.splitlines() if ln.startswith("{")]) == 1
    p = _run("bench.start_deadline(100, 1, 1)\n"
             "bench.HEADLINE.update(rec={'metric': 'm'}, t=time.time(), rank=1)\ntime.sleep(30)")
    assert p.returncode == 0
    assert p.stdout.strip() == ""
