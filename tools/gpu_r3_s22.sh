#!/bin/bash
# Round 3 session 22: the 8-rank pipelined host-staging stall of session 14 with at most 2
# hardware queues per process (16 in all) against the default 4 (up to 32): is it the same
# queue oversubscription that slows config 5 (profiles/r3_s21_queues)?
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r3_s22"
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {
  local tag=$1; shift
  local n=$1; shift
  timeout -k 10 120 python -m rabit_amd.launcher -n "$n" --timeout 100 -- python tools/host_stage_probe.py "$@" \
    > "$OUT/run.log" 2>&1
  local rc=$?
  grep -h '"probe"' "$OUT/run.log" | sed "s/^/$tag /" | tee -a "$OUT/probe.txt" | cut -c1-500
  if [ $rc -ne 0 ]; then tail -20 "$OUT/run.log"; echo "stopping rc=$rc"; exit $rc; fi
}
run q4 8 rabit_host_stage_chunk=0
run q4 8 rabit_host_stage_chunk=16M rabit_host_stage_streams=3
export GPU_MAX_HW_QUEUES=2
run q2 8 rabit_host_stage_chunk=0
run q2 8 rabit_host_stage_chunk=16M rabit_host_stage_streams=3
run q2 8 rabit_host_stage_chunk=16M rabit_host_stage_streams=1
