#!/bin/bash
# Round 3 session 24: what the second-destination deferral protects.  Rank 1 dies in the middle
# of a multi-chunk device allreduce (mock_die_mid) with the deferral on (default) and off
# (rabit_device_defer_second=0, the behaviour before it): off, the survivors retry with part of
# their input already overwritten by the first chunk's result and the model misses its closed
# form.  Pull form, 3 ranks sharing the GPU.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r3_s24"
mkdir -p "$OUT"
export TMPDIR=/tmp
for defer in 1 0; do
  echo "== defer_second=$defer"
  timeout -k 10 200 python -m rabit_amd.launcher -n 3 --num-attempt 2 --timeout 180 -- \
    python tests/scripts/device_ft.py mock_die_mid=1,1,0,0 rabit_device_direct_mode=pull \
    rabit_device_fused=0 rabit_device_defer_second=$defer > "$OUT/defer_$defer.log" 2>&1
  rc=$?
  echo "rc=$rc"
  grep -h "DEVFT OK\|Die Mid Op\|AssertionError\|resumed" "$OUT/defer_$defer.log" | cut -c1-200 | head -12
  if [ $rc -eq 124 ] || [ $rc -eq 137 ]; then echo "timed out: stopping"; exit $rc; fi
done
