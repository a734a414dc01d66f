# round 6: the RNS small-batch decrypt (k_dec_rns) - parity first, then the A/B against k_dec_wave
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r6f}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  -k "decrypt" > $OUT/tests_dec.log 2>&1; rc=$?
tail -5 $OUT/tests_dec.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  XHE_DEC_RNS=0 timeout -k 10 200 python -u tools/dec_shapes.py 1 15 64 256 512 >> $OUT/dec_wave.jsonl 2>> $OUT/dec.err || exit 3
  timeout -k 10 200 python -u tools/dec_shapes.py 1 15 64 256 512 >> $OUT/dec_rns.jsonl 2>> $OUT/dec.err || exit 3
done
cat $OUT/dec_wave.jsonl $OUT/dec_rns.jsonl | cut -c1-400
timeout -k 10 300 python -u tools/lr_he_demo.py --epochs 3 --cpu-batches 0 --sync-phases > $OUT/lr_sync.json 2> $OUT/lr_sync.err || { tail -5 $OUT/lr_sync.err; exit 3; }
tail -c 1200 $OUT/lr_sync.json
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_dropin.py tests/test_gpu_lr_demo.py \
  tests/test_gpu_shapes.py tests/test_gpu_codec.py tests/test_gpu_matvec.py > $OUT/tests.log 2>&1; rc=$?
tail -4 $OUT/tests.log
exit $rc
