#!/bin/bash
# Round 3 session 31: barriers numbered on the device and the graphable direct allreduce: the
# new multi-rank graph test first, then the whole GPU suite (every barrier of every form
# changed), smoke() and the N=1 bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r3_s31"
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
  local name=$1; shift
  local limit=$1; shift
  echo "== $name"
  timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  grep -h "GRAPHDIRECT OK\|passed\|failed" "$OUT/$name.log" | tail -4 | cut -c1-300 || true
  if [ $rc -ne 0 ]; then tail -40 "$OUT/$name.log"; echo "stopping: $name rc=$rc"; exit $rc; fi
}
step pytest_graph 300 python -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_engine.py -x -v -s -p no:cacheprovider --timeout 200 --timeout-method thread -k "graphable"
step pytest_gpu 1000 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_n1 300 python bench.py --steps 20 --warmup 5
