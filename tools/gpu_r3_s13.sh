#!/bin/bash
# Round 3 session 13: pipelined host staging (host buffers through HBM).  GPU tests of the
# host-via-device path (whole copies and the pipelined stager), then the reference's own
# speed_test against xrabit's, 128 MiB float32 host buffers, N = 2 / 4 / 8 on the box's GPU.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r3_s13"
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
  local name=$1; shift
  local limit=$1; shift
  echo "== $name"
  timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -4 "$OUT/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then tail -30 "$OUT/$name.log"; echo "stopping: $name rc=$rc"; exit $rc; fi
}
step pytest_hostdev 400 python -u -m pytest tests/test_gpu_multirank.py -x -v -p no:cacheprovider --timeout 200 --timeout-method thread -k "host_buffers_via_device or direct_recovery"
step h2h 900 python tools/refbuild/compare_speed.py --worlds 2 4 8 --n 33554432 --nrep 3 --impl reference xrabit_via_dev_whole xrabit_via_dev --out "$OUT/h2h.jsonl"
