#!/bin/bash
# Round 3 session 18: the driver's scaling launches (N = 2, 4, 8 under torch.distributed.run,
# --steps 20 --warmup 5) on the current tree, every rank sharing the box's one GPU: the bench
# contract end to end, host-buffer extra included.  Not an xGMI measurement.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r3_s18"
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
  local name=$1; shift
  local limit=$1; shift
  echo "== $name"
  local t0=$(date +%s)
  timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc wall=$(( $(date +%s) - t0 ))s"
  grep -h '^{' "$OUT/$name.log" | tail -1 | cut -c1-400 || true
  if [ $rc -ne 0 ]; then tail -30 "$OUT/$name.log"; echo "stopping: $name rc=$rc"; exit $rc; fi
}
for n in 2 4 8; do
  step torchrun_n$n 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29740 + n)) bench.py --gpus $n --steps 20 --warmup 5
done
