set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -k graphable -x -v -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/graphar.log 2>&1; rc=$?; tail -15 gpurun_out/graphar.log; exit $rc
