#!/bin/bash
# Round 3 session 39: the whole GPU suite, smoke(), the N=1 bench with its rocprofv3 kernel
# statistics, and the driver's N = 2 / 4 / 8 launches (ranks sharing the GPU) on the tree with
# the pipelined push allreduce, the folded tail copy and the link probe.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r3_s39"
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
  local name=$1; shift
  local limit=$1; shift
  echo "== $name"
  timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  grep -h '^{' "$OUT/$name.log" | tail -1 | cut -c1-300 || true
  tail -2 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then tail -40 "$OUT/$name.log"; echo "stopping: $name rc=$rc"; exit $rc; fi
}
step pytest_gpu 1000 python -u -m pytest tests -m gpu -x -q -s -p no:cacheprovider --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_n1 300 python bench.py --steps 20 --warmup 5
for n in 2 4 8; do
  step torchrun_n$n 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29930 + n)) bench.py --gpus $n --steps 20 --warmup 5
done
