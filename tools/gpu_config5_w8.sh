#!/bin/bash
# BASELINE config 5 at its specified 8 ranks, all sharing the box's one GPU (a semantics and
# cost rehearsal, not an xGMI measurement): no failure, then rank 3 killed at version 4.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/c5w8"
mkdir -p "$OUT"
export TMPDIR=/tmp
XR_ITERS=12 timeout -k 10 240 python -m rabit_amd.launcher -n 8 --num-attempt 1 --timeout 220 -- \
  python tools/robust_bench.py > "$OUT/rb_w8_clean.log" 2>&1 || { tail -20 "$OUT/rb_w8_clean.log"; exit 1; }
grep ROBUST "$OUT/rb_w8_clean.log" | head -2
XR_ITERS=12 timeout -k 10 240 python -m rabit_amd.launcher -n 8 --num-attempt 2 --timeout 220 -- \
  python tools/robust_bench.py mock=3,4,0,0 > "$OUT/rb_w8_kill.log" 2>&1 || { tail -20 "$OUT/rb_w8_kill.log"; exit 1; }
grep ROBUST "$OUT/rb_w8_kill.log" | head -2
