set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 120 ./build/bin/d2h_probe > gpurun_out/d2h_probe.log 2>&1; rc=$?; cat gpurun_out/d2h_probe.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/d2hprof -o d2h -- ./build/bin/d2h_probe > gpurun_out/d2h_prof.log 2>&1; rc=$?; tail -3 gpurun_out/d2h_prof.log; exit $rc
