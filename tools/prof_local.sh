#!/bin/bash
# Kernel + memory-copy trace of device-resident local checkpoints (tests/scripts/device_local.py)
# with 3 ranks sharing the GPU, each rank under its own rocprofv3 (ranks started by this shell;
# the tracker runs in rank 0, rabit_amd/torchrun.py).  Shows how the local replicas move:
# device copy kernels of the direct transport, no host staging.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/prof_local"
mkdir -p "$OUT"
export PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}" TMPDIR=/tmp MASTER_ADDR=127.0.0.1 MASTER_PORT=29710 WORLD_SIZE=3 LOCAL_WORLD_SIZE=3 XR_ENV_INIT=1
pids=()
for r in 0 1 2; do
  RANK=$r LOCAL_RANK=$r timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --stats \
    --output-format csv -d "$OUT/r$r" -o local -- python3 tests/scripts/device_local.py \
    > "$OUT/rank$r.log" 2>&1 &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait "$p" || rc=$?; done
grep -h "DEVLOCAL" "$OUT"/rank*.log || true
exit $rc
