# round 6: per-stream workspace lists - parity across the ops that take workspaces, then the streams A/B
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r6s}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_serialize_pipeline.py tests/test_gpu_resident.py tests/test_gpu_dropin.py > $OUT/tests.log 2>&1; rc=$?
tail -n 3 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for cfg in "1 524288" "2 262144" "2 524288"; do
    set -- $cfg
    XHE_ENC_STREAMS=$1 XHE_ENC_SUB=$2 timeout -k 10 200 python -u tools/enc_ser_rates.py 2>> $OUT/err.log | sed "s/^{/{\"streams\": $1, /" >> $OUT/enc_ser.jsonl || exit 3
  done
done
cat $OUT/enc_ser.jsonl
