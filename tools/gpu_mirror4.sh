set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
MIRROR_SETTINGS=0:off,0,0:engine=sdma,0:engine=sdma:off timeout -k 10 300 python -u tools/mirror_probe.py > gpurun_out/mirror_probe4.log 2>&1 || { tail -30 gpurun_out/mirror_probe4.log; exit 1; }
cat gpurun_out/mirror_probe4.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_recovery.py -k "mirror_copy" -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/mirror4_tests.log 2>&1; rc=$?; tail -3 gpurun_out/mirror4_tests.log; exit $rc
