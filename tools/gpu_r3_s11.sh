#!/bin/bash
# Round 3 session 11: the whole GPU suite on the tree with the pipelined direct broadcast and
# the broadcast calibration, smoke(), the N=1 bench, and a kernel trace of the pipelined
# broadcast with 4 ranks sharing the GPU (each rank under its own rocprofv3).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r3_s11"
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
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -s -p no:cacheprovider --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_n1 300 python bench.py --steps 20 --warmup 5
# 4 ranks sharing the GPU, each under its own rocprofv3: the automatic pipeline chunk, then one
# chunk (the unpipelined round structure)
prof_w4() {
  local tag=$1 chunk=$2 port=$3
  export MASTER_ADDR=127.0.0.1 MASTER_PORT=$port WORLD_SIZE=4 LOCAL_WORLD_SIZE=4
  local pids=() rc=0
  for r in 0 1 2 3; do
    RANK=$r LOCAL_RANK=$r timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$OUT/prof_bcast_$tag/r$r" -o bcast -- python3 tools/bcast_probe.py "$chunk" \
      > "$OUT/prof_bcast_${tag}_rank$r.log" 2>&1 &
    pids+=($!)
  done
  for p in "${pids[@]}"; do wait "$p" || rc=$?; done
  echo "== prof_bcast_$tag rc=$rc"
  grep -h '^{' "$OUT"/prof_bcast_${tag}_rank*.log || tail -20 "$OUT/prof_bcast_${tag}_rank0.log"
  return $rc
}
prof_w4 auto 0 29652 && prof_w4 one_chunk 268435456 29662
