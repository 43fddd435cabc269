set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/graphar -o base -- python3 -m rabit_amd.launcher -n 1 -- python3 tests/scripts/graph_allreduce.py base > gpurun_out/graphar_prof.log 2>&1; rc=$?; grep -h "GRAPHAR" gpurun_out/graphar_prof.log; cut -d, -f1-4 gpurun_out/graphar/*kernel_stats.csv 2>/dev/null | cut -c1-160 | head -12; exit $rc
