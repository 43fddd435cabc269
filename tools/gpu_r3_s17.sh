#!/bin/bash
# Round 3 session 17: the whole GPU suite on the tree with pipelined host staging, smoke(), the
# N=1 bench and its rocprofv3 kernel statistics.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r3_s17"
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
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -s -p no:cacheprovider --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_n1 300 python bench.py --steps 20 --warmup 5
step prof_n1 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_n1" -o bench -- python3 bench.py --steps 20 --warmup 5
