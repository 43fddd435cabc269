#!/bin/bash
# Round 3 session 28: the guarded tail copy folded into the last gather launch: multi-rank GPU
# tests of every direct form, then per-form 128 MiB robust allreduce kernel traces (2 ranks).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r3_s28"
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_multirank.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "push or recovery or death or half or direct_collectives or calibration or small_op or link_probe" > "$OUT/pytest.log" 2>&1
rc=$?
tail -2 "$OUT/pytest.log"
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" "$OUT/pytest.log" | head -20; exit $rc; fi
export MASTER_ADDR=127.0.0.1 WORLD_SIZE=2 LOCAL_WORLD_SIZE=2
prof() {
  local mode=$1 port=$2
  export MASTER_PORT=$port
  local pids=() rc=0
  for r in 0 1; do
    RANK=$r LOCAL_RANK=$r timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$OUT/$mode/r$r" -o k -- python3 tools/pipeline_probe.py "$mode" \
      > "$OUT/${mode}_rank$r.log" 2>&1 &
    pids+=($!)
  done
  for p in "${pids[@]}"; do wait "$p" || rc=$?; done
  echo "== $mode rc=$rc"
  grep -h '^{' "$OUT"/${mode}_rank*.log || tail -20 "$OUT/${mode}_rank0.log"
  return $rc
}
prof pipelined 29841 && prof push 29851 && prof pull 29861
