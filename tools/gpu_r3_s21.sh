#!/bin/bash
# Round 3 session 21: BASELINE config 5's phases at 8 and 4 ranks sharing the GPU
# (tools/config5_probe.py), to find why the 256 MiB iteration is 20x slower at 8 ranks.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r3_s21"
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
  local name=$1; shift
  local limit=$1; shift
  echo "== $name"
  timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  grep -h '^{' "$OUT/$name.log" | cut -c1-900 || true
  if [ $rc -ne 0 ]; then tail -30 "$OUT/$name.log"; echo "stopping: $name rc=$rc"; exit $rc; fi
}
# first call: step w8 (default queues), step w4
#step w8 240 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29791 tools/config5_probe.py
# second call: the same 8 ranks with at most 2 hardware queues per process (16 in all)
export GPU_MAX_HW_QUEUES=2
step w8_q2 240 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29793 tools/config5_probe.py
