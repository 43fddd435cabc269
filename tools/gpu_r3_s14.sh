#!/bin/bash
# Round 3 session 14: where the time of a pipelined host-buffer allreduce goes (2, 4 and 8 ranks
# sharing the box's GPU): whole copies, three streams, one stream.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r3_s14"
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {
  local n=$1; shift
  timeout -k 10 120 python -m rabit_amd.launcher -n "$n" --timeout 100 -- python tools/host_stage_probe.py "$@" \
    > "$OUT/run.log" 2>&1
  local rc=$?
  grep -h '"probe"' "$OUT/run.log" | tee -a "$OUT/probe.jsonl" | cut -c1-600
  if [ $rc -ne 0 ]; then tail -20 "$OUT/run.log"; echo "stopping rc=$rc"; exit $rc; fi
}
for n in 2 4 8; do
  run $n rabit_host_stage_chunk=0
  run $n rabit_host_stage_chunk=16M rabit_host_stage_streams=3
  run $n rabit_host_stage_chunk=16M rabit_host_stage_streams=1
  run $n rabit_host_stage_chunk=32M rabit_host_stage_streams=1
done
