#!/bin/bash
# Round 3 session 20 (second call: robust engine): 8 ranks sharing the GPU, direct allreduce from 64 to 256 MiB with per-phase
# hipEvent timing (which phase grows past 128 MiB), against 4 ranks.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r3_s20"
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
  local name=$1; shift
  local limit=$1; shift
  echo "== $name"
  timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  grep -h '^{' "$OUT/$name.log" | cut -c1-400 || true
  if [ $rc -ne 0 ]; then tail -30 "$OUT/$name.log"; echo "stopping: $name rc=$rc"; exit $rc; fi
}
export XR_SIZES=67108864,134217728,201326592,268435456 XR_PHASE=1 XR_FUSED=0 XR_REPS=5
export XR_LIB=standard
step w8 240 python -m rabit_amd.launcher -n 8 --num-attempt 1 --timeout 220 -- python tools/direct_bench.py
