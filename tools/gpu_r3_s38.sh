#!/bin/bash
# Round 3 session 38: the pipelined-form tests after the chunk clamp.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r3_s38"
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_multirank.py -x -v -p no:cacheprovider --timeout 250 --timeout-method thread -k "pipelined or calibration or link_probe or graphable" > "$OUT/pytest.log" 2>&1
rc=$?
grep -E "PASSED|FAILED|passed|failed" "$OUT/pytest.log" | tail -20
exit $rc
