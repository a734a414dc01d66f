# round 6: per-chunk timeline of the serialize pipeline over a running encryption
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r6q}; mkdir -p $OUT
for sub in 1048576 262144; do
  XHE_PIPE_TRACE=1 XHE_ENC_SUB=$sub timeout -k 10 200 python -u tools/enc_ser_rates.py >> $OUT/enc_ser.jsonl 2>> $OUT/trace_$sub.err || exit 3
done
cat $OUT/enc_ser.jsonl
tail -n 2 $OUT/trace_1048576.err | cut -c1-1500
tail -n 2 $OUT/trace_262144.err | cut -c1-1500
