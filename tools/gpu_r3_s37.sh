#!/bin/bash
# Round 3 session 37: BASELINE config 5 at its 8 ranks on the final tree (device-numbered
# barriers, second-destination deferral): clean, and with rank 3 killed after version 4
# (tools/robust_bench.py under the repo launcher; ranks share the box's GPU).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r3_s37"
mkdir -p "$OUT"
export TMPDIR=/tmp XR_ITERS=12
step() {
  local name=$1; shift
  local limit=$1; shift
  echo "== $name"
  timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  grep -h "summary\|restart_to_loaded" "$OUT/$name.log" | cut -c1-400 | head -4
  grep -c '"ok": true' "$OUT/$name.log"
  if [ $rc -ne 0 ]; then tail -30 "$OUT/$name.log"; echo "stopping: $name rc=$rc"; exit $rc; fi
}
step c5w8_clean 240 python -m rabit_amd.launcher -n 8 --num-attempt 1 --timeout 220 -- python tools/robust_bench.py
step c5w8_kill 240 python -m rabit_amd.launcher -n 8 --num-attempt 2 --timeout 220 -- python tools/robust_bench.py mock=3,4,0,0
