#!/bin/bash
# Round 3 session 27: kernel traces of the pipelined push allreduce against the classic push
# form, 2 ranks sharing the GPU, each rank under its own rocprofv3 (robust engine, 128 MiB).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r3_s27"
mkdir -p "$OUT"
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1 WORLD_SIZE=2 LOCAL_WORLD_SIZE=2
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
prof pipelined 29821 && prof push 29831
