#!/bin/bash
# The one GPU-box session runner (replaces the per-session scripts of earlier rounds; the named
# sessions that produced round 4's evidence are in tools/gpu_next_session.sh).
#
#   OUT_NAME=r4_xyz STEPS="tests smoke bench1 shared" bash tools/gpu_run.sh
#
# Every step that touches the GPU runs under its own `timeout -k 10`, output goes to
# gpurun_out/$OUT_NAME/<step>.log, and any non-zero exit ends the session (no retries), so a
# fault, abort or time limit never starts another GPU step in the same call.
#
# Steps:
#   tests     pytest -m gpu (whole GPU suite, one process)
#   gtest     pytest -m gpu -k "$GPU_K" (a subset)
#   gfiles    pytest -m gpu over the files $GPU_FILES (the suite split over two calls)
#   smoke     __graft_entry__.smoke()
#   bench1    bench.py at N=1 (the driver's 1-GPU run)
#   shared    the driver's N = $SHARED_NS launches (torchrun, every rank on this box's one GPU)
#   prof      rocprofv3 --kernel-trace --stats of the N=1 bench
#   kbench    kernel bench against the measured HBM peak
#   robust    tools/robust_bench.py = BASELINE config 5 on $ROBUST_N (8) shared ranks: clean, then
#             rank 3 killed at version 4 (restarted by the launcher), recovery phase breakdown;
#             ROBUST_REPS=k repeats the kill run (robust_kill_<i>.log)
#   zctrace   tools/zero_copy_trace.sh: kernel order with / without the zero-copy registry
#   cmd       an arbitrary command: CMD="..." (limit CMD_LIMIT seconds, default 300)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/${OUT_NAME:-session}"
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
  local name=$1; shift
  local limit=$1; shift
  echo "== $name (limit ${limit}s) $(date +%T)"
  timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc $(date +%T)"
  grep -h '^{' "$OUT/$name.log" | tail -1 | cut -c1-400 || true
  tail -3 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then tail -40 "$OUT/$name.log"; echo "stopping: $name rc=$rc"; exit $rc; fi
}
PYT="python -u -m pytest -x -q -s -p no:cacheprovider --timeout 300 --timeout-method thread --durations=25"
for s in ${STEPS:-tests smoke bench1}; do
  case $s in
    tests)  step pytest_gpu 1100 $PYT tests -m gpu ;;
    gtest)  step pytest_gpu_k 900 $PYT tests -m gpu -k "${GPU_K:?set GPU_K}" ;;
    gfiles) step pytest_gpu_files 1000 $PYT ${GPU_FILES:?set GPU_FILES} -m gpu ;;
    gtestf) step pytest_gpu_fk 1000 $PYT ${GPU_FILES:?set GPU_FILES} -m gpu -k "${GPU_K:?set GPU_K}" ;;
    smoke)  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench1) step bench_n1 300 python bench.py --steps ${STEPS_K:-20} --warmup 5 ;;
    shared)
      for n in ${SHARED_NS:-2 4 8}; do
        step torchrun_n$n 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
          --master-addr 127.0.0.1 --master-port $((29930 + n)) bench.py --gpus $n \
          --steps ${STEPS_K:-20} --warmup 5 ${BENCH_ARGS:-}
      done ;;
    prof)   step rocprof 400 rocprofv3 --kernel-trace --stats --output-format csv \
              -d "$OUT/prof" -o bench -- python3 bench.py --steps 10 --warmup 3 ;;
    kbench) step kbench 300 python tools/kernel_bench.py ;;
    robust)
      step robust_clean 260 env XR_ITERS=12 python -m rabit_amd.launcher -n ${ROBUST_N:-8} \
        --num-attempt 1 --timeout 240 -- python -u tools/robust_bench.py ${ROBUST_ARGS:-}
      for rep in $(seq 1 ${ROBUST_REPS:-1}); do
        sfx=$([ "${ROBUST_REPS:-1}" = 1 ] || echo "_$rep")
        step robust_kill$sfx 260 env XR_ITERS=12 python -m rabit_amd.launcher -n ${ROBUST_N:-8} \
          --num-attempt 2 --timeout 240 -- python -u tools/robust_bench.py mock=3,4,0,0 \
          ${ROBUST_ARGS:-}
      done ;;
    zctrace) step zctrace 300 bash tools/zero_copy_trace.sh ;;
    cmd)    step cmd 600 bash -c "${CMD:?set CMD}" ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "session done"
