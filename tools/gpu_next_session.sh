# The next GPU-box session; argv[1] picks it.
#   s8: smoke, the N=1 bench, the driver-shaped N = 2 / 4 / 8 launches (ranks share the GPU)
#   s9: calibrated N=4 bench (size sweep), zero-copy kernel trace, device allgather with and
#       without the on-device layout, BASELINE config 5 at 8 ranks with the rank-3 kill
set -u
case ${1:-s8} in
  s7b)
    # the GPU tests after the one that stalled in r4_s7, then s8
    OUT_NAME=r4_s7b GPU_K="calibration_flow or symmetric_zero_copy or registered_zero_copy or gradient_buckets or bench_torchrun_shared_gpu or direct_half_precision or device_local_checkpoint_recovery or device_hang_detected or forced_rccl_on_shared or rccl_init_failure_falls_back or small_op_stress or rccl_lifecycle or test_gpu_recovery or test_recovery" \
      STEPS="gtest" bash tools/gpu_run.sh || exit $?
    OUT_NAME=r4_s8 STEPS="smoke bench1 shared" bash tools/gpu_run.sh ;;
  s8) OUT_NAME=r4_s8 STEPS="smoke bench1 shared" bash tools/gpu_run.sh ;;
  s9)
    OUT_NAME=r4_s9 STEPS="zctrace" bash tools/gpu_run.sh || exit $?
    OUT_NAME=r4_s9 CMD="python -m rabit_amd.launcher -n 4 -- python -u tests/scripts/allgather_resolved.py && python -m rabit_amd.launcher -n 4 -- python -u tests/scripts/allgather_resolved.py rabit_device_allgather_resolve=0" \
      STEPS="cmd" bash tools/gpu_run.sh || exit $?
    OUT_NAME=r4_s9 STEPS="robust" bash tools/gpu_run.sh ;;
  s10)
    # recovery with the exit pipe (sockets shut and the launcher told before _Exit), then the
    # GPU fault-tolerance tests that restart workers through the launcher
    OUT_NAME=r4_s10 STEPS="robust" bash tools/gpu_run.sh || exit $?
    OUT_NAME=r4_s10 GPU_K="chaos or recover or hang or device_ft or mock or kill or adopts" \
      STEPS="gtest" bash tools/gpu_run.sh ;;
  s11)
    # the checkpoint-route fix (a device-loaded rank relays on the TCP route), calibration
    OUT_NAME=r4_s11 GPU_K="chaos or recover or hang or device_ft or mock or kill or adopts or calibration" \
      STEPS="gtest" bash tools/gpu_run.sh ;;
  s12a)
    OUT_NAME=r4_s12a GPU_FILES="tests/test_bench_contract.py tests/test_gpu_device_reducer.py tests/test_gpu_engine.py tests/test_gpu_kernels.py tests/test_gpu_models.py" \
      STEPS="gfiles smoke bench1 prof" bash tools/gpu_run.sh ;;
  s12b)
    OUT_NAME=r4_s12b GPU_FILES="tests/test_gpu_multirank.py tests/test_gpu_rccl_lifecycle.py tests/test_gpu_recovery.py tests/test_recovery.py" \
      STEPS="gfiles shared" bash tools/gpu_run.sh ;;
  s13)
    # a slow headline after the suite: what holds the GPU after the hang tests?
    timeout -k 10 120 python tools/hbm_probe.py start || exit $?
    OUT_NAME=r4_s13 GPU_K="device_hang_detected" STEPS="gtest" bash tools/gpu_run.sh || exit $?
    timeout -k 10 120 python tools/hbm_probe.py after_hang_tests || exit $?
    sleep 5
    timeout -k 10 120 python tools/hbm_probe.py after_5s || exit $?
    OUT_NAME=r4_s13 SHARED_NS=2 STEPS="shared" bash tools/gpu_run.sh || exit $?
    timeout -k 10 120 python tools/hbm_probe.py end ;;
  s14)
    # the multirank tests s7b did not run (s8's benches after s7b were fine, s12b's after the
    # whole file were not), then what holds the GPU, then the N=2 bench
    OUT_NAME=r4_s14 GPU_FILES="tests/test_gpu_multirank.py" GPU_K="not (calibration_flow or symmetric_zero_copy or registered_zero_copy or gradient_buckets or bench_torchrun_shared_gpu or direct_half_precision or device_local_checkpoint_recovery or device_hang_detected or forced_rccl_on_shared or rccl_init_failure_falls_back or small_op_stress)" \
      STEPS="gtestf" bash tools/gpu_run.sh || exit $?
    timeout -k 10 120 python tools/hbm_probe.py after_tests || exit $?
    OUT_NAME=r4_s14 SHARED_NS=2 STEPS="shared" bash tools/gpu_run.sh || exit $?
    timeout -k 10 120 python tools/hbm_probe.py end ;;
  s15)
    # the rest of s12b's set (s14 ran the first part): multirank tests s7b also ran, RCCL
    # lifecycle, recovery; then what holds the GPU, then the N=2 bench
    OUT_NAME=r4_s15 GPU_FILES="tests/test_gpu_multirank.py tests/test_gpu_rccl_lifecycle.py tests/test_gpu_recovery.py tests/test_recovery.py" GPU_K="calibration_flow or symmetric_zero_copy or registered_zero_copy or gradient_buckets or bench_torchrun_shared_gpu or direct_half_precision or device_local_checkpoint_recovery or device_hang_detected or forced_rccl_on_shared or rccl_init_failure_falls_back or small_op_stress or rccl_lifecycle or test_gpu_recovery or test_recovery" \
      STEPS="gtestf" bash tools/gpu_run.sh || exit $?
    timeout -k 10 120 python tools/hbm_probe.py after_tests || exit $?
    OUT_NAME=r4_s15 SHARED_NS=2 STEPS="shared" bash tools/gpu_run.sh || exit $?
    timeout -k 10 120 python tools/hbm_probe.py end ;;
  s16)
    # the bench with a checkpoint before its timed loop; the bench's own GPU tests
    OUT_NAME=r4_s16 GPU_K="bench" STEPS="gtest smoke bench1 shared" bash tools/gpu_run.sh ;;
  s17)
    # peers' barriers poisoned by the rank that sees a failure first (kPeerAbortOffset): the
    # recovery breakdown, then the fault-tolerance GPU tests
    OUT_NAME=r4_s17 STEPS="robust" bash tools/gpu_run.sh || exit $?
    OUT_NAME=r4_s17 GPU_K="chaos or recover or hang or device_ft or mock or kill or adopts or calibration or direct_collectives" \
      STEPS="gtest" bash tools/gpu_run.sh ;;
  s18)
    # the recovery breakdown, three kill runs (eight ranks time-slicing one GPU vary run to run)
    OUT_NAME=r4_s18 ROBUST_REPS=3 STEPS="robust" bash tools/gpu_run.sh ;;
  s19)
    # A/B on one box: the peer abort on (default) and off, three kill runs each
    OUT_NAME=r4_s19 ROBUST_REPS=3 STEPS="robust" bash tools/gpu_run.sh || exit $?
    OUT_NAME=r4_s19_nopa ROBUST_REPS=3 ROBUST_ARGS="rabit_device_peer_abort=0" STEPS="robust" \
      bash tools/gpu_run.sh ;;
  s20)
    # A/B again with the abort passed on by the barrier kernel itself (no stream per group)
    OUT_NAME=r4_s20 ROBUST_REPS=3 STEPS="robust" bash tools/gpu_run.sh || exit $?
    OUT_NAME=r4_s20_nopa ROBUST_REPS=3 ROBUST_ARGS="rabit_device_peer_abort=0" STEPS="robust" \
      bash tools/gpu_run.sh ;;
  s21a)
    OUT_NAME=r4_s21a GPU_FILES="tests/test_bench_contract.py tests/test_gpu_device_reducer.py tests/test_gpu_engine.py tests/test_gpu_kernels.py tests/test_gpu_models.py" \
      STEPS="gfiles smoke bench1 prof" bash tools/gpu_run.sh ;;
  s21b)
    OUT_NAME=r4_s21b GPU_FILES="tests/test_gpu_multirank.py tests/test_gpu_rccl_lifecycle.py tests/test_gpu_recovery.py tests/test_recovery.py" \
      STEPS="gfiles shared" bash tools/gpu_run.sh ;;
  s22)
    # ExitProcess without allocation: the fault-tolerance GPU tests and one config-5 kill run
    OUT_NAME=r4_s22 GPU_K="chaos or recover or hang or device_ft or mock or kill or adopts or rccl_lifecycle or test_recovery" \
      STEPS="gtest robust" bash tools/gpu_run.sh ;;
  s23)
    # the whole GPU suite in one call, as the driver runs it at round end, then smoke
    OUT_NAME=r4_s23 STEPS="tests smoke" bash tools/gpu_run.sh ;;
esac
