set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for m in plain xwait after lowprio; do
  timeout -k 10 60 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/d2hmodes -o $m -- ./build/bin/d2h_modes $m > gpurun_out/d2hmodes_$m.log 2>&1 || { tail -5 gpurun_out/d2hmodes_$m.log; exit 1; }
  echo "$m: blit=$(grep -c copyBuffer gpurun_out/d2hmodes/${m}_kernel_trace.csv 2>/dev/null) sdma=$(grep -c DEVICE_TO_HOST gpurun_out/d2hmodes/${m}_memory_copy_trace.csv 2>/dev/null)"
done
