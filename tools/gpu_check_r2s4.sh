set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_recovery.py -k mirror_copy -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r2s4_mirror_test.log 2>&1; rc=$?; tail -4 gpurun_out/r2s4_mirror_test.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 200 --warmup 10 --extras 0 > gpurun_out/r2s4_bench200.log 2>&1; rc=$?; grep '^{' gpurun_out/r2s4_bench200.log | cut -c1-300; exit $rc
