#!/bin/bash
# Round 3 session 10: pipelined direct broadcast + broadcast calibration.  Multi-rank direct
# tests (ranks share the GPU), world-1 transports, N=1 bench, 4-rank torchrun rehearsal.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r3_s10"
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
step pytest_bcast 600 python -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_engine.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "direct_collectives or world1 or broadcast or bcast"
step bench_n1 300 python bench.py --steps 20 --warmup 5
step torchrun_n4 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29711 bench.py --gpus 4 --steps 5 --warmup 2
