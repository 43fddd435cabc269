set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
MIRROR_SETTINGS=0,0:low,16:low,64:low timeout -k 10 300 python -u tools/mirror_probe.py > gpurun_out/mirror_probe3.log 2>&1 || { tail -30 gpurun_out/mirror_probe3.log; exit 1; }
cat gpurun_out/mirror_probe3.log
