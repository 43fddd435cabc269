"""Summarise rocprofv3 --pmc counter CSVs (tools/gpu_session.sh step `pmc`) per kernel.

    python tools/pmc_summary.py gpurun_out/pmc/fetch_counter_collection.csv \
        gpurun_out/pmc/write_counter_collection.csv > profiles/<run>/pmc_summary.json

For every kernel (name shortened to 90 characters): the mean of each counter over its
dispatches, plus the mean duration.  FETCH_SIZE / WRITE_SIZE are in KiB as rocprofv3 reports
them; GRBM_GUI_ACTIVE is GPU busy cycles.
"""
import csv
import json
import sys
from collections import defaultdict


def main(paths):
    acc = defaultdict(lambda: defaultdict(list))
    for p in paths:
        with open(p, newline="") as f:
            for row in csv.DictReader(f):
                name = row["Kernel_Name"][:90]
                acc[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
                dur = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3
                acc[name]["duration_us"].append(dur)
    out = {}
    for name, counters in acc.items():
        out[name] = {k: round(sum(v) / len(v), 3) for k, v in counters.items()}
    json.dump(out, sys.stdout, indent=1, sort_keys=True)
    print()


if __name__ == "__main__":
    main(sys.argv[1:])
