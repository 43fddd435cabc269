# zero-copy registry diagnosis (2 ranks sharing the GPU), then the new GPU tests
set -u
mkdir -p gpurun_out/r4_s6
echo "== zc debug $(date +%T)"
timeout -k 10 100 python -m rabit_amd.launcher -n 2 -- python -u tests/scripts/zero_copy_check.py rabit_debug=1 rabit_device_peer_timeout_sec=10 > gpurun_out/r4_s6/zc.log 2>&1
rc=$?
echo "zc rc=$rc"; grep -m5 "gave up" gpurun_out/r4_s6/zc.log; tail -5 gpurun_out/r4_s6/zc.log
[ $rc -ne 0 ] && exit $rc
OUT_NAME=r4_s6 GPU_K="zero_copy or allgather_layout or calibration or host_stage_auto or rccl_lifecycle or symmetric" STEPS="gtest" bash tools/gpu_run.sh
