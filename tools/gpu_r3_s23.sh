#!/bin/bash
# Round 3 session 23: the pipelined push allreduce (ar_plan.h) and the second-destination
# deferral of multi-chunk ops: GPU tests (forms, recovery, a death inside a multi-chunk op,
# calibration, half precision, the bench contract), then the direct transport's 128 MiB
# allreduce per form with 2, 4 and 8 ranks sharing the GPU.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r3_s23"
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
  local name=$1; shift
  local limit=$1; shift
  echo "== $name"
  timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  grep -h '^{' "$OUT/$name.log" | cut -c1-300 || true
  tail -3 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then tail -40 "$OUT/$name.log"; echo "stopping: $name rc=$rc"; exit $rc; fi
}
step pytest_pipe 900 python -u -m pytest tests/test_gpu_multirank.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "push or recovery or death or half or calibration or bench_torchrun"
export XR_SIZES=4194304,33554432,134217728 XR_FUSED=0 XR_REPS=7
for n in 2 4 8; do
  step db_pull_w$n 240 python -m rabit_amd.launcher -n $n --num-attempt 1 --timeout 220 -- python tools/direct_bench.py rabit_device_direct_mode=pull
  step db_push_w$n 240 python -m rabit_amd.launcher -n $n --num-attempt 1 --timeout 220 -- python tools/direct_bench.py rabit_device_direct_mode=push
  step db_pipe_w$n 240 python -m rabit_amd.launcher -n $n --num-attempt 1 --timeout 220 -- python tools/direct_bench.py rabit_device_direct_mode=pipelined
done
