#!/bin/bash
# Round 3 session 6: fused vs classic at world 1 (no phase events in the timed pass) and with 2
# ranks sharing the GPU; grid variant at world 1; RCCL-path fused prepare under rocprof.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r3_s6"
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
step fused_w1_g2048 120 python3 tools/fused_w1_bench.py --sizes 16M,128M --reps 30 --forms fused --port 9394 rabit_device_fused_grid=2048
step fused_w1_g512 120 python3 tools/fused_w1_bench.py --sizes 16M,128M --reps 30 --forms fused --port 9395 rabit_device_fused_grid=512
XR_SIZES=4194304,16777216,134217728 XR_FUSED=0 step w2_classic 240 python3 -m rabit_amd.launcher -n 2 -- python3 tools/direct_bench.py
XR_SIZES=4194304,16777216,134217728 XR_FUSED=1 step w2_fused 240 python3 -m rabit_amd.launcher -n 2 -- python3 tools/direct_bench.py
step prep_rccl_w1 120 python3 tools/prep_rccl_w1.py
step prep_rccl_prof 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prep_prof" -o prep -- python3 tools/prep_rccl_w1.py
