# round 6: rows per encryption launch under the serialize pipeline (same box, alternating)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r6o}; mkdir -p $OUT
for r in 1 2; do
  for sub in 1048576 524288 262144 131072; do
    XHE_ENC_SUB=$sub timeout -k 10 200 python -u tools/enc_ser_rates.py >> $OUT/enc_ser.jsonl 2>> $OUT/enc_ser.err || exit 3
  done
done
cat $OUT/enc_ser.jsonl
