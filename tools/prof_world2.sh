#!/bin/bash
# Kernel profile of a 2-rank bench on one GPU box: each rank runs under its own rocprofv3
# (ranks started by this shell, not by torchrun, so no process hop sits between the profiler and
# python).  Outside torchrun the tracker binds MASTER_PORT + 17 (rabit_amd/torchrun.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/prof_w2"
mkdir -p "$OUT"
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1 MASTER_PORT=29650 WORLD_SIZE=2 LOCAL_WORLD_SIZE=2
pids=()
for r in 0 1; do
  RANK=$r LOCAL_RANK=$r timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$OUT/r$r" -o bench -- python3 bench.py --gpus 2 --steps 10 --warmup 3 \
    > "$OUT/rank$r.log" 2>&1 &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait "$p" || rc=$?; done
grep -h '^{' "$OUT"/rank*.log || true
exit $rc
