#!/bin/bash
# GPU-box session used this round: GPU tests, reference-vs-xrabit speed_test head-to-head
# (128 MiB float32, host TCP and HBM), bench + rocprofv3 kernel stats.  Each step has its own
# limit; a crash/timeout stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out"; mkdir -p "$OUT"; export TMPDIR=/tmp
step() {
  local name=$1; shift; local limit=$1; shift
  echo "== $name"; timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "== $name rc=$rc"; tail -4 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then echo "stopping at $name"; exit $rc; fi
}
for s in ${STEPS:-tests h2h prof}; do
  case $s in
    tests) step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    h2h) step h2h 900 python -u tools/refbuild/compare_speed.py --worlds 1 2 4 8 --n 33554432 --nrep 3 --out "$OUT/h2h.jsonl" ;;
    bench) step bench 600 python bench.py --steps 20 --warmup 5 ;;
    prof) step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o bench -- python3 bench.py --steps 10 --warmup 3 ;;
  esac
done
echo "session done"
