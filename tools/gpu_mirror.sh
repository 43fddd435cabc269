# host-mirror cost vs the overlapped step (tools/mirror_probe.py), a kernel trace of the narrow
# mirror, then the GPU tests that recover from mirrored checkpoints
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u tools/mirror_probe.py > gpurun_out/mirror_probe.log 2>&1 || { tail -30 gpurun_out/mirror_probe.log; exit 1; }
cat gpurun_out/mirror_probe.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/mirrorprof -o m16 -- python3 tools/mirror_probe.py 16 > gpurun_out/mirror_prof.log 2>&1 || { tail -20 gpurun_out/mirror_prof.log; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_recovery.py tests/test_gpu_models.py tests/test_gpu_engine.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/mirror_tests.log 2>&1; rc=$?; tail -3 gpurun_out/mirror_tests.log; exit $rc
