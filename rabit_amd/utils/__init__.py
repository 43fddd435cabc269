"""Small helpers around the native library: timing, trace merging, parameter strings.

The reference's utility layer is C++ (`include/rabit/internal/{utils,timer}.h`, mirrored in
csrc/include/rabit/internal); these are the Python-side conveniences for jobs and tools.
"""
from __future__ import annotations

import json
import os
import time
from typing import Dict, Iterable, List


class Timer:
    """Wall-clock accumulator (rabit::utils::GetTime equivalent), usable as a context manager."""

    def __init__(self):
        self.total = 0.0
        self.count = 0
        self._t0 = None

    def __enter__(self):
        self._t0 = time.perf_counter()
        return self

    def __exit__(self, *exc):
        self.total += time.perf_counter() - self._t0
        self.count += 1
        return False

    @property
    def mean(self) -> float:
        return self.total / self.count if self.count else 0.0


def params_to_args(**params) -> List[str]:
    """{'rabit_debug': 1} -> ['rabit_debug=1'] (the argv form rabit.init / rabit::Init take)."""
    return ["%s=%s" % (k, v) for k, v in params.items()]


def merge_traces(paths: Iterable[str], out: str) -> int:
    """Merge per-rank Chrome traces written by rabit_amd.dump_trace (rabit_trace=1) into one file
    that chrome://tracing / Perfetto shows with one process row per rank.  Returns the number of
    events written."""
    events: List[Dict] = []
    for p in paths:
        with open(p) as f:
            data = json.load(f)
        evs = data["traceEvents"] if isinstance(data, dict) else data
        events.extend(evs)
    events.sort(key=lambda e: e.get("ts", 0))
    tmp = out + ".tmp"
    with open(tmp, "w") as f:
        json.dump({"traceEvents": events, "displayTimeUnit": "us"}, f)
    os.replace(tmp, out)
    return len(events)


def summarize_trace(path: str) -> Dict[str, Dict[str, float]]:
    """Per span name: count, total and mean duration (us) of a Chrome trace from dump_trace."""
    with open(path) as f:
        data = json.load(f)
    evs = data["traceEvents"] if isinstance(data, dict) else data
    out: Dict[str, Dict[str, float]] = {}
    for e in evs:
        if e.get("ph") != "X":
            continue
        s = out.setdefault(e["name"], {"count": 0, "total_us": 0.0})
        s["count"] += 1
        s["total_us"] += float(e.get("dur", 0.0))
    for s in out.values():
        s["mean_us"] = s["total_us"] / s["count"]
    return out


__all__ = ["Timer", "params_to_args", "merge_traces", "summarize_trace"]
