# round 6: serialize pipeline with a copy-only stream (bit lengths from the rows on the host)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r6p}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_serialize_pipeline.py \
  tests/test_gpu_codec.py > $OUT/tests.log 2>&1; rc=$?
tail -n 3 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for sub in 1048576 262144 131072; do
    XHE_ENC_SUB=$sub timeout -k 10 200 python -u tools/enc_ser_rates.py >> $OUT/enc_ser.jsonl 2>> $OUT/enc_ser.err || exit 3
  done
done
cat $OUT/enc_ser.jsonl
