set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
MIRROR_SETTINGS=0,0:sdma,256,1024 timeout -k 10 300 python -u tools/mirror_probe.py > gpurun_out/mirror_probe2.log 2>&1 || { tail -30 gpurun_out/mirror_probe2.log; exit 1; }
cat gpurun_out/mirror_probe2.log
HSA_ENABLE_SDMA=1 timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/mirrorprof2 -o sdma -- python3 tools/mirror_probe.py 0 > gpurun_out/mirror_prof2.log 2>&1 || { tail -20 gpurun_out/mirror_prof2.log; exit 1; }
grep -c copyBuffer gpurun_out/mirrorprof2/sdma_kernel_trace.csv || true
