#!/bin/bash
# Round 3 session 5: fused vs classic at world 1 after the reduce/gather unroll, small-op
# breakdown, bench contract (busbw + config 5), direct-transport multi-rank tests (dual-store
# broadcast / allgather, recovery).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r3_s5"
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
  local name=$1; shift
  local limit=$1; shift
  echo "== $name"
  timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  grep -h '^{' "$OUT/$name.log" || tail -25 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then tail -40 "$OUT/$name.log"; echo "stopping: $name rc=$rc"; exit $rc; fi
}
step fused_w1 240 python3 tools/fused_w1_bench.py --sizes 1M,4M,16M,128M --reps 30
step small_op_w2 180 python3 -m rabit_amd.launcher -n 2 -- python3 tools/small_op_probe.py 4096
step small_op_w1 120 python3 -m rabit_amd.launcher -n 1 -- python3 tools/small_op_probe.py 4096 rabit_world1_fastpath=0 rabit_device_world1_transport=1
step multirank 900 python -u -m pytest tests/test_gpu_multirank.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "direct_collectives or direct_recovery or bench_torchrun"
step contract 400 python -u -m pytest tests/test_bench_contract.py -x -v -s -p no:cacheprovider --timeout 360 --timeout-method thread
step prep_rccl_w1 120 python3 tools/prep_rccl_w1.py
step prep_rccl_prof 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prep_prof" -o prep -- python3 tools/prep_rccl_w1.py
