#!/bin/bash
# Round 3 session 32: the graphable direct allreduce with a barrier on each side: its GPU tests,
# then base-engine allreduces over the direct transport, eager against captured into one
# hipGraph (2 and 4 ranks sharing the GPU).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r3_s32"
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_engine.py -x -v -p no:cacheprovider --timeout 200 --timeout-method thread -k "graphable" > "$OUT/pytest.log" 2>&1
rc=$?
tail -1 "$OUT/pytest.log"
if [ $rc -ne 0 ]; then tail -30 "$OUT/pytest.log"; exit $rc; fi
for n in 2 4; do
  timeout -k 10 200 python -m rabit_amd.launcher -n $n --num-attempt 1 --timeout 180 -- python tools/graph_direct_bench.py > "$OUT/w$n.log" 2>&1
  rc=$?
  echo "== w$n rc=$rc"
  grep -h '^{' "$OUT/w$n.log" || tail -20 "$OUT/w$n.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
