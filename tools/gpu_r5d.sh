bash tools/gpu_round.sh r5d tests bench || exit $?
for r in 1 2; do
  RATES_ONLY=pub,add,sum bash tools/gpu_round.sh r5d rates && RATES_ONLY=pub,add RATES_ENV="XHE_ADD_BAR=0" bash tools/gpu_round.sh r5d rates || exit 3
done
O=gpurun_out/r5d
XHE_LIB=$PWD/xfl_amd/lib/dev8192.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shapes.py tests/test_gpu_dropin.py -k 8192 -v --timeout 600 --timeout-method thread > $O/tests8192.log 2>&1
rc=$?; tail -5 $O/tests8192.log; if [ $rc -gt 1 ]; then exit $rc; fi
for r in 1 2; do
  timeout -k 10 400 python -u tools/bench_keysizes.py --bits 8192 >> $O/ks8192_main.jsonl 2>> $O/ks.err || exit 3
  XHE_LIB=$PWD/xfl_amd/lib/dev8192.so timeout -k 10 400 python -u tools/bench_keysizes.py --bits 8192 >> $O/ks8192_dev.jsonl 2>> $O/ks.err || exit 3
done
cat $O/ks8192_main.jsonl $O/ks8192_dev.jsonl | cut -c1-300
