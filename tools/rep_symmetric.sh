# repeat the symmetric zero-copy check (ranks share the GPU) to catch intermittent failures
W=${W:-3}
for i in 1 2 3 4 5 6 7 8; do
  timeout -k 10 60 python -m rabit_amd.launcher -n $W --timeout 50 python tests/scripts/symmetric_check.py $EXTRA > gpurun_out/rep_$i.log 2>&1
  rc=$?
  echo "iter $i rc=$rc $(grep -c 'SYMMETRIC OK' gpurun_out/rep_$i.log) ok; $(grep -h AssertionError gpurun_out/rep_$i.log | head -2)"
done
