#!/bin/bash
# Round 3 session 33: kernel trace of the graphed 4 KiB direct allreduce (2 ranks sharing the
# GPU, each under its own rocprofv3): where a replayed op's 80 us go.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r3_s33"
mkdir -p "$OUT"
export TMPDIR=/tmp XR_SIZES=4096
timeout -k 10 200 python -m rabit_amd.launcher -n 2 --num-attempt 1 --timeout 180 -- rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof_%pid%" -o k -- python3 tools/graph_direct_bench.py > "$OUT/w2.log" 2>&1
rc=$?
echo "rc=$rc"
grep -h '^{' "$OUT/w2.log" || tail -20 "$OUT/w2.log"
ls "$OUT"
exit $rc
