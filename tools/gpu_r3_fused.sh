#!/bin/bash
# Round 3: fused vs classic direct two-shot at world 1 (no CU sharing), timed and under a
# rocprofv3 kernel trace per form.  Every GPU step has its own limit; a crash stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r3_fused_w1"
mkdir -p "$OUT"
export TMPDIR=/tmp
SIZES=${SIZES:-1M,4M,16M,128M}
run() {
  local name=$1; shift
  echo "== $name"
  timeout -k 10 240 "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  grep -h '^{' "$OUT/$name.log" || tail -20 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then echo "stopping: $name rc=$rc"; exit $rc; fi
}
run timing python3 tools/fused_w1_bench.py --sizes "$SIZES" --reps 30 ${EXTRA:-}
run prof_classic rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_classic" \
  -o classic -- python3 tools/fused_w1_bench.py --sizes "$SIZES" --reps 10 --forms classic --port 9392 ${EXTRA:-}
run prof_fused rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_fused" \
  -o fused -- python3 tools/fused_w1_bench.py --sizes "$SIZES" --reps 10 --forms fused --port 9393 ${EXTRA:-}
