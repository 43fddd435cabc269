#!/bin/bash
# Round 3 session 19: why BASELINE config 5 slows down 20x from 4 to 8 ranks on the shared GPU.
# Hypothesis: hardware-queue oversubscription.  The host-buffer extra (just before config 5)
# creates the pipelined stager's two extra streams in every rank; 8 processes x 4 queues exceed
# what the GPU maps at once.  Same launch with the stager never created (rabit_host_stage=0)
# and with its copies on the plane stream (rabit_host_stage_streams=1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r3_s19"
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
  local name=$1; shift
  local limit=$1; shift
  echo "== $name"
  timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  grep -h '^{' "$OUT/$name.log" | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['extras']; print({k: e[k] for k in e if k.startswith('config5') or k.startswith('checkpoint') or k.startswith('host_buffer')})" || true
  if [ $rc -ne 0 ]; then tail -30 "$OUT/$name.log"; echo "stopping: $name rc=$rc"; exit $rc; fi
}
step n8_default 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29761 bench.py --gpus 8 --steps 20 --warmup 5 --variants 0
export rabit_host_stage=0
step n8_no_stager 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29771 bench.py --gpus 8 --steps 20 --warmup 5 --variants 0
unset rabit_host_stage
export rabit_host_stage_streams=1
step n8_one_stream 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29781 bench.py --gpus 8 --steps 20 --warmup 5 --variants 0
