#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r3_s4"
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 5 90 ./build/bin/rccl_lifecycle_test > "$OUT/lifecycle.log" 2>&1
rc=$?
echo "lifecycle rc=$rc"
grep -v "Could not read node\|^$" "$OUT/lifecycle.log" | tail -40
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -m pytest tests/test_gpu_rccl_lifecycle.py -x -v -s -p no:cacheprovider --timeout 180 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?
echo "pytest rc=$rc"
tail -30 "$OUT/pytest.log"
exit $rc
