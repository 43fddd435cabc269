set -u
export TMPDIR=/tmp
OUT=gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "recover or ckpt or checkpoint or models or engine" > $OUT/ck_tests.log 2>&1 || { tail -30 $OUT/ck_tests.log; exit 1; }
tail -2 $OUT/ck_tests.log
for m in idle always; do
  XR_ITERS=12 timeout -k 10 200 python -m rabit_amd.launcher -n 4 --num-attempt 1 --timeout 180 -- python tools/robust_bench.py rabit_device_ckpt_mirror=$m > $OUT/rb_$m.log 2>&1 || { tail -20 $OUT/rb_$m.log; exit 1; }
  grep -h "ROBUST" $OUT/rb_$m.log | head -1 | cut -c1-600
done
XR_ITERS=12 timeout -k 10 200 python -m rabit_amd.launcher -n 4 --num-attempt 2 --timeout 180 -- python tools/robust_bench.py mock=3,4,0,0 > $OUT/rb_kill.log 2>&1 || { tail -20 $OUT/rb_kill.log; exit 1; }
grep -h "ROBUST" $OUT/rb_kill.log | head -1 | cut -c1-600
