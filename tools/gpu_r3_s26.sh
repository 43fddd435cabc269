#!/bin/bash
# Round 3 session 26: rabit.link_probe() (GPU test), and bench.py at N = 2 and 8 under the
# driver's launch with the probe in its extras (ranks share the GPU: HBM, not xGMI, here).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r3_s26"
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
  local name=$1; shift
  local limit=$1; shift
  echo "== $name"
  timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  grep -h "link probe:\|passed\|failed" "$OUT/$name.log" | tail -3 | cut -c1-400 || true
  grep -h '^{' "$OUT/$name.log" | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d.get('post_headline_failure'), d['transport']['calibration_forms_us'], (d.get('extras') or {}).get('link_probe_min_over_ranks'))" 2>/dev/null || true
  if [ $rc -ne 0 ]; then tail -40 "$OUT/$name.log"; echo "stopping: $name rc=$rc"; exit $rc; fi
}
step pytest_probe 300 python -u -m pytest tests/test_gpu_multirank.py -x -v -s -p no:cacheprovider --timeout 200 --timeout-method thread -k "link_probe"
step torchrun_n2 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29801 bench.py --gpus 2 --steps 20 --warmup 5
step torchrun_n8 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29808 bench.py --gpus 8 --steps 20 --warmup 5
