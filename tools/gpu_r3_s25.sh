#!/bin/bash
# Round 3 session 25: the whole GPU suite after the pipelined allreduce and the second-destination
# deferral (fused kernels now leave the user buffer to the guarded copy), smoke(), the N=1 bench,
# and the 4 KiB robust allreduce at 2 ranks (the fused one-shot plus its guarded copy).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r3_s25"
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
  local name=$1; shift
  local limit=$1; shift
  echo "== $name"
  timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  grep -h '^{' "$OUT/$name.log" | tail -2 | cut -c1-400 || true
  tail -3 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then tail -40 "$OUT/$name.log"; echo "stopping: $name rc=$rc"; exit $rc; fi
}
step small_op_w2 180 python3 -m rabit_amd.launcher -n 2 -- python3 tools/small_op_probe.py 4096
step pytest_gpu 1000 python -u -m pytest tests -m gpu -x -q -s -p no:cacheprovider --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_n1 300 python bench.py --steps 20 --warmup 5
