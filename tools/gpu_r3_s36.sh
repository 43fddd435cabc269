#!/bin/bash
# Round 3 session 36: bench.py at N=2 (driver launch, ranks sharing the GPU) after the link probe
# was isolated in the extras.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r3_s36"
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29911 bench.py --gpus 2 --steps 20 --warmup 5 > "$OUT/n2.log" 2>&1
rc=$?
echo "rc=$rc"
grep -h '^{' "$OUT/n2.log" | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['extras']; print(d['value'], d.get('post_headline_failure'), e.get('link_probe_min_over_ranks'), e.get('busbw_over_all_links_read'), e.get('link_probe_error'))"
exit $rc
