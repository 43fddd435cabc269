# checkpoint_tensors cost at world 1: plain timing, then a rocprofv3 kernel + HIP runtime trace
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 120 python tools/ckpt_probe.py 12 > gpurun_out/ck_plain.log 2>&1 || { tail gpurun_out/ck_plain.log; exit 1; }
grep checkpoint_ gpurun_out/ck_plain.log
timeout -k 10 240 rocprofv3 --kernel-trace --hip-runtime-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/ckprof -o ck -- python3 tools/ckpt_probe.py 12 > gpurun_out/ck_prof.log 2>&1 || { tail gpurun_out/ck_prof.log; exit 1; }
grep checkpoint_ gpurun_out/ck_prof.log
