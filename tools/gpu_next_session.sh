set -u
mkdir -p gpurun_out/r4_s3
echo "== zc debug $(date +%T)"
timeout -k 10 150 python -m rabit_amd.launcher -n 2 -- python -u tests/scripts/zero_copy_check.py rabit_debug=1 rabit_device_peer_timeout_sec=10 > gpurun_out/r4_s3/zc2.log 2>&1
rc=$?
echo "zc rc=$rc"; tail -30 gpurun_out/r4_s3/zc2.log
[ $rc -ne 0 ] && exit $rc
OUT_NAME=r4_s3 GPU_K="zero_copy or allgather_layout or calibration or host_stage_auto or rccl_lifecycle or symmetric" STEPS="gtest" bash tools/gpu_run.sh
