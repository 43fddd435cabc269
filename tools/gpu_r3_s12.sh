#!/bin/bash
# Round 3 session 12: the driver's N=8 launch rehearsed on the current tree (8 ranks sharing the
# GPU), and BASELINE config 5 at 8 ranks (clean, then rank 3 killed at version 4 and recovered).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r3_s12"
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
  local name=$1; shift
  local limit=$1; shift
  echo "== $name"
  timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  grep -h '^{' "$OUT/$name.log" | tail -2 | cut -c1-600 || true
  if [ $rc -ne 0 ]; then tail -30 "$OUT/$name.log"; echo "stopping: $name rc=$rc"; exit $rc; fi
}
step torchrun_n8 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29720 bench.py --gpus 8 --steps 5 --warmup 2
export XR_ITERS=12
step c5w8_clean 240 python -m rabit_amd.launcher -n 8 --num-attempt 1 --timeout 220 -- python tools/robust_bench.py
grep -h ROBUST "$OUT/c5w8_clean.log" | head -2 | cut -c1-400
step c5w8_kill 240 python -m rabit_amd.launcher -n 8 --num-attempt 2 --timeout 220 -- python tools/robust_bench.py mock=3,4,0,0
grep -h ROBUST "$OUT/c5w8_kill.log" | head -2 | cut -c1-400
