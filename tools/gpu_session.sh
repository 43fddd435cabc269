#!/bin/bash
# One GPU-box session: GPU tests, 1-GPU bench, rocprofv3 kernel profile.
# Every GPU step has its own time limit; a crash/timeout (rc >= 124) stops the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out"
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
  local name=$1; shift
  local limit=$1; shift
  echo "== $name (limit ${limit}s)"
  timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -5 "$OUT/$name.log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
    echo "stopping: $name ended with rc=$rc"; exit $rc
  fi
}
STEPS=${STEPS:-"tests bench prof"}
for s in $STEPS; do
  case $s in
    tests) step pytest_gpu 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider ;;
    bench) step bench 600 python bench.py --steps 20 --warmup 5 ;;
    prof)  step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv \
             -d "$OUT/prof" -o bench -- python3 bench.py --steps 10 --warmup 3 ;;
    multi) step multi 900 python -u -m pytest tests/test_gpu_multirank.py -x -v -p no:cacheprovider \
             --timeout 300 --timeout-method thread \
             -k "${MULTI_K:-}" ;;
    ktests) step ktests 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -p no:cacheprovider \
             --timeout 120 --timeout-method thread ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    kbench) step kbench 300 python tools/kernel_bench.py ;;
    kprof) step kprof 300 rocprofv3 --kernel-trace --stats --output-format csv \
             -d "$OUT/kprof" -o kbench -- python3 tools/kernel_bench.py --reps 5 --rounds 1 --inner 2 ;;
    pmc) step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv \
             -d "$OUT/pmc" -o fetch -- python3 tools/kernel_bench.py --reps 3 --rounds 1 &&
         step pmc_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv \
             -d "$OUT/pmc" -o write -- python3 tools/kernel_bench.py --reps 3 --rounds 1 ;;
    dbench)
      # direct transport on ranks sharing the GPU: fused (one launch per chunk) vs classic
      for w in 2 4; do
        for mode in pull push; do
          for f in 1 0; do
            XR_FUSED=$f step dbench_w${w}_${mode}_f$f 300 python -m rabit_amd.launcher -n $w -- \
              python tools/direct_bench.py rabit_device_direct_mode=$mode
          done
        done
      done ;;
    profw2) step profw2 400 bash tools/prof_world2.sh ;;
    proflocal) step proflocal 300 bash tools/prof_local.sh ;;
    speed) step speed 300 python -m rabit_amd.launcher -n 1 -- build/bin/speed_test 33554432 10 device=1 rabit_world1_fastpath=0 ;;
  esac
done
echo "session done"
