#!/bin/bash
# Round 3 session 8: the whole GPU suite, the N=1 bench, and a kernel profile of 4 ranks sharing
# the GPU (bench extras: broadcast dual store, config 5).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r3_s8"
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
  local name=$1; shift
  local limit=$1; shift
  echo "== $name"
  timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  grep -h '^{' "$OUT/$name.log" | tail -3 || true
  tail -4 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then echo "stopping: $name rc=$rc"; exit $rc; fi
}
step pytest_gpu 800 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread
step bench_n1 300 python bench.py --steps 20 --warmup 5
