#!/bin/bash
# Round 3 session 35: the graphed direct allreduce with ONE process (a one-rank direct group,
# rabit_device_world1_transport=1): if its replayed kernels run in a few us, the 50 us kernels of
# session 33 come from two processes sharing the GPU, not from graph replay itself.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r3_s35"
mkdir -p "$OUT"
export TMPDIR=/tmp XR_SIZES=4096,1048576
timeout -k 10 200 python -m rabit_amd.launcher -n 1 --num-attempt 1 --timeout 180 -- rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof_%pid%" -o k -- python3 tools/graph_direct_bench.py rabit_world1_fastpath=0 rabit_device_world1_transport=1 rabit_device_algo=direct > "$OUT/w1.log" 2>&1
rc=$?
echo "rc=$rc"
grep -h '^{' "$OUT/w1.log" || tail -20 "$OUT/w1.log"
exit $rc
