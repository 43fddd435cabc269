# Named GPU-box sessions of round 4 (each drives tools/gpu_run.sh; gpurun runs one at a time):
#   gpurun --timeout 1200 -- 'bash tools/gpu_next_session.sh final'
#   final     the whole GPU suite in one call (as the driver runs it) and smoke  -> r4_final/
#   headline  smoke, the N=1 bench, the driver-shaped N = 2 / 4 / 8 launches   -> r4_final/
#   evidence  calibrated N=4 bench, zero-copy kernel trace, device allgather with and without the
#             host round                       -> r4_calibration/, r4_zero_copy/, r4_allgather/
#   recovery  config 5 at 8 ranks with the rank-3 kill, 3 runs each with the peer abort on and
#             off                                                               -> r4_recovery/
#   ft        the fault-tolerance GPU tests (chaos, recovery, hangs, kills, RCCL lifecycle)
#   zc        the zero-copy and allgather GPU tests, then the N=2 launch
set -u
case ${1:-final} in
  final) OUT_NAME=r4_final_suite STEPS="tests smoke" bash tools/gpu_run.sh ;;
  headline) OUT_NAME=r4_headline STEPS="smoke bench1 shared" bash tools/gpu_run.sh ;;
  evidence)
    OUT_NAME=r4_evidence SHARED_NS=4 XRABIT_PARAMS=rabit_device_calibrate_test=1 STEPS="shared" \
      bash tools/gpu_run.sh || exit $?
    OUT_NAME=r4_evidence STEPS="zctrace" bash tools/gpu_run.sh || exit $?
    OUT_NAME=r4_evidence CMD="python -m rabit_amd.launcher -n 4 -- python -u tests/scripts/allgather_resolved.py && python -m rabit_amd.launcher -n 4 -- python -u tests/scripts/allgather_resolved.py rabit_device_allgather_resolve=0" \
      STEPS="cmd" bash tools/gpu_run.sh ;;
  recovery)
    OUT_NAME=r4_recovery_on ROBUST_REPS=3 STEPS="robust" bash tools/gpu_run.sh || exit $?
    OUT_NAME=r4_recovery_off ROBUST_REPS=3 ROBUST_ARGS="rabit_device_peer_abort=0" STEPS="robust" \
      bash tools/gpu_run.sh ;;
  ft)
    OUT_NAME=r4_ft GPU_K="chaos or recover or hang or device_ft or mock or kill or adopts or rccl_lifecycle or test_recovery" \
      STEPS="gtest" bash tools/gpu_run.sh ;;
  zc)
    OUT_NAME=r4_zc GPU_K="zero_copy or symmetric or allgather_layout or calibration_flow or expandable" \
      STEPS="gtest" bash tools/gpu_run.sh || exit $?
    OUT_NAME=r4_zc SHARED_NS=2 STEPS="shared" bash tools/gpu_run.sh ;;
  *) echo "unknown session $1"; exit 2 ;;
esac
