#!/bin/bash
# Round 3 session 2: RCCL lifecycle GPU tests, then fused vs classic at world 1 again.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r3_s2"
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
  local name=$1; shift
  local limit=$1; shift
  echo "== $name"
  timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -25 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then echo "stopping: $name rc=$rc"; exit $rc; fi
}
step lifecycle 240 python -u -m pytest tests/test_gpu_rccl_lifecycle.py -x -v -s -p no:cacheprovider --timeout 200 --timeout-method thread
step fused_w1 240 python3 tools/fused_w1_bench.py --sizes 1M,4M,16M,128M --reps 30
step small_op_w2 180 python3 -m rabit_amd.launcher -n 2 -- python3 tools/small_op_probe.py 4096
step contract 400 python -u -m pytest tests/test_bench_contract.py -x -v -s -p no:cacheprovider --timeout 360 --timeout-method thread
