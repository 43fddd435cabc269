#!/usr/bin/env python3
"""Summarise repeated config-5 kill runs (`tools/gpu_run.sh` step `robust` with ROBUST_REPS):
per run, rank 0's summary and restart timeline and the survivors' detect phase; then the medians.

    python tools/robust_summary.py gpurun_out/r4_s18/robust_kill_*.log
"""
import json
import re
import statistics
import sys


def runs(paths):
    dec = json.JSONDecoder()
    for path in paths:
        text = open(path, encoding="utf-8", errors="replace").read()
        recs = []
        for m in re.finditer(r"ROBUST ", text):
            try:
                rec, _ = dec.raw_decode(text[m.end():])
            except ValueError:
                continue
            recs.append(rec)
        r0 = [r for r in recs if r["rank"] == 0 and "summary" in r]
        if not r0:
            continue
        s = r0[0]["summary"]
        tl = s.get("restart_timeline_ms", {})
        restarted = [r for r in recs if r.get("attempt", 0) > 0]
        survivors = [r for r in recs if r.get("attempt", 0) == 0]
        yield {
            "log": path,
            "models_ok": all(r["model_check"]["ok"] for r in recs) and len(recs) >= 8,
            "failure_iter_ms": s["failure_iter_ms_max_over_ranks"],
            "minus_startup_ms": s["failure_iter_minus_startup_ms"],
            "minus_restart_to_loaded_ms": round(
                s["failure_iter_ms_max_over_ranks"] -
                1e3 * restarted[0]["restart_to_loaded_s"], 1) if restarted else None,
            "detect_ms_median_survivors": round(statistics.median(
                r["recovery_phases_s"]["detect"] * 1e3 for r in survivors), 1),
            "init_to_loaded_ms": tl.get("init_to_checkpoint_loaded"),
            "restarted_first_iteration_ms": tl.get("restarted_first_iteration"),
            "steady_iter_ms": s["steady_iter_ms_median"],
        }


def main():
    rows = list(runs(sys.argv[1:]))
    for r in rows:
        print(json.dumps(r))
    if rows:
        keys = [k for k in rows[0] if k not in ("log", "models_ok")]
        med = {k: statistics.median(r[k] for r in rows if r[k] is not None) for k in keys}
        print("median over %d runs: %s" % (len(rows), json.dumps(med)))
        print("all models exact:", all(r["models_ok"] for r in rows))


if __name__ == "__main__":
    main()
