#!/bin/bash
# Round 3 session 9: kernel bench (roof normalised to the run's peak), 4 ranks sharing the GPU
# under per-rank rocprofv3 (bench extras: dual-store broadcast, config 5), 8-rank torchrun
# rehearsal of the driver's N=8 launch.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r3_s9"
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
  local name=$1; shift
  local limit=$1; shift
  echo "== $name"
  timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  grep -h '^{' "$OUT/$name.log" | tail -30 || true
  if [ $rc -ne 0 ]; then tail -30 "$OUT/$name.log"; echo "stopping: $name rc=$rc"; exit $rc; fi
}
step kbench 300 python3 tools/kernel_bench.py
# 4 ranks, each under its own profiler (no process hop between rocprofv3 and python)
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29650 WORLD_SIZE=4 LOCAL_WORLD_SIZE=4
pids=()
for r in 0 1 2 3; do
  RANK=$r LOCAL_RANK=$r timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$OUT/prof_w4/r$r" -o bench -- python3 bench.py --gpus 4 --steps 3 --warmup 1 --variants 0 \
    > "$OUT/prof_w4_rank$r.log" 2>&1 &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait "$p" || rc=$?; done
echo "== prof_w4 rc=$rc"
grep -h '^{' "$OUT"/prof_w4_rank*.log || tail -20 "$OUT/prof_w4_rank0.log"
[ $rc -eq 0 ] || exit $rc
unset MASTER_ADDR MASTER_PORT WORLD_SIZE LOCAL_WORLD_SIZE
step torchrun_n8 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29710 bench.py --gpus 8 --steps 5 --warmup 2
