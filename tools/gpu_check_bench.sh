set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_multirank.py -k "bench_torchrun" -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/g2_pytest.log 2>&1; rc=$?; tail -4 gpurun_out/g2_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 8 --steps 10 --warmup 3 > gpurun_out/g2_n8.log 2>&1; rc=$?; grep '^{' gpurun_out/g2_n8.log | cut -c1-600; [ $rc -ne 0 ] && { tail -20 gpurun_out/g2_n8.log; exit $rc; }
timeout -k 10 200 python -m rabit_amd.launcher -n 2 -- python examples/basic.py > gpurun_out/g2_basic.log 2>&1; rc=$?; cat gpurun_out/g2_basic.log | tail -6; exit $rc
