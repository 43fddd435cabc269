#!/bin/bash
# lifecycle test alone, with RCCL's own log, to see where it stops
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r3_s3"
mkdir -p "$OUT"
export TMPDIR=/tmp
NCCL_DEBUG=INFO NCCL_DEBUG_SUBSYS=INIT,BOOTSTRAP timeout -k 5 60 ./build/bin/rccl_lifecycle_test > "$OUT/lifecycle.log" 2>&1
rc=$?
echo "rc=$rc"
tail -60 "$OUT/lifecycle.log"
exit $rc
