set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 120 python3 tools/d2h_torch_modes.py envdiff 2>&1 | grep envdiff || true
run() {  # name mode [env...]
  local name=$1 m=$2; shift 2
  timeout -k 10 120 env "$@" rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/d2htorch -o $name -- python3 tools/d2h_torch_modes.py $m > gpurun_out/d2htorch_$name.log 2>&1 || { tail -5 gpurun_out/d2htorch_$name.log; exit 1; }
  echo "$name: blit=$(grep -c copyBuffer gpurun_out/d2htorch/${name}_kernel_trace.csv 2>/dev/null) sdma=$(grep -c DEVICE_TO_HOST gpurun_out/d2htorch/${name}_memory_copy_trace.csv 2>/dev/null)"
}
run torchlib torchlib X=1
run hip_forceblit0 hip GPU_FORCE_BLIT_COPY_SIZE=0
run hip_sdmaon hip HSA_ENABLE_SDMA=1 HSA_ENABLE_SDMA_COPY_SIZE_OVERRIDE=1
