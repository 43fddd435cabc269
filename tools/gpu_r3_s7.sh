#!/bin/bash
# fused two-shot: L2-invalidating acquire vs ordering-only acquire (world 1 and 2 shared ranks);
# small-op probe with the kernel-written completion word
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r3_s7"
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
XRABIT_FUSED_LIGHT=1 step fused_w1_light 240 python3 tools/fused_w1_bench.py --sizes 4M,16M,128M --reps 30 --forms fused
XRABIT_FUSED_LIGHT=1 XR_SIZES=4194304,16777216,134217728 XR_FUSED=1 step w2_fused_light 240 python3 -m rabit_amd.launcher -n 2 -- python3 tools/direct_bench.py
step small_op_w2 180 python3 -m rabit_amd.launcher -n 2 -- python3 tools/small_op_probe.py 4096
step small_op_w2_event 180 python3 -m rabit_amd.launcher -n 2 -- python3 tools/small_op_probe.py 4096 rabit_device_done_word=0
step small_op_w1 120 python3 -m rabit_amd.launcher -n 1 -- python3 tools/small_op_probe.py 4096 rabit_world1_fastpath=0 rabit_device_world1_transport=1
step multirank 600 python -u -m pytest tests/test_gpu_multirank.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "direct_collectives"
