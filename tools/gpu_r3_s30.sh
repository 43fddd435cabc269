#!/bin/bash
# Round 3 session 30: the roctx ranges of the tracing subsystem (rabit_trace_roctx=1) in a
# rocprofv3 marker + kernel trace: 2 ranks sharing the GPU, each under its own rocprofv3, a few
# robust allreduces, a broadcast and a checkpoint (tools/pipeline_probe.py's op, traced).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r3_s30"
mkdir -p "$OUT"
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1 WORLD_SIZE=2 LOCAL_WORLD_SIZE=2 MASTER_PORT=29891
export rabit_trace_roctx=1 rabit_trace=1
pids=()
rc=0
for r in 0 1; do
  RANK=$r LOCAL_RANK=$r timeout -k 10 240 rocprofv3 --marker-trace --kernel-trace --output-format csv \
    -d "$OUT/r$r" -o t -- python3 tools/pipeline_probe.py pull > "$OUT/rank$r.log" 2>&1 &
  pids+=($!)
done
for p in "${pids[@]}"; do wait "$p" || rc=$?; done
echo "rc=$rc"
grep -h '^{' "$OUT"/rank*.log || tail -20 "$OUT/rank0.log"
ls "$OUT"/r0
exit $rc
