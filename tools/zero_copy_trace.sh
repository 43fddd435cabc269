#!/bin/bash
# Kernel order of the direct pull two-shot with and without the zero-copy registry, 2 ranks
# sharing this box's GPU, each rank under its own rocprofv3 --kernel-trace (ranks started by this
# shell: no process hop between the profiler and python).  See tools/zero_copy_trace.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/${OUT_NAME:-zc_trace}/trace"
mkdir -p "$OUT"
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1 MASTER_PORT=29670 WORLD_SIZE=2 LOCAL_WORLD_SIZE=2
pids=()
for r in 0 1; do
  RANK=$r LOCAL_RANK=$r timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv \
    -d "$OUT/r$r" -o zc -- python3 tools/zero_copy_trace.py > "$OUT/rank$r.log" 2>&1 &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait "$p" || rc=$?; done
[ $rc -ne 0 ] && { tail -n 20 "$OUT"/rank*.log; exit $rc; }
for r in 0 1; do
  csvf=$(find "$OUT/r$r" -name '*kernel_trace.csv' | head -1)
  python3 tools/zero_copy_trace.py --analyze "$csvf" "$OUT/rank$r.log" "$OUT/rank${r}_ops.json" \
    || exit 1
done
