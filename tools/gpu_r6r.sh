# round 6: pieces of the pipelined encryption on one or two streams (the pool
# allocator blocks the host when a piece's workspace was freed on the other stream)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r6r}; mkdir -p $OUT
for r in 1 2; do
  for cfg in "1 1048576" "1 524288" "1 262144" "2 262144"; do
    set -- $cfg
    XHE_PIPE_TRACE=1 XHE_ENC_STREAMS=$1 XHE_ENC_SUB=$2 timeout -k 10 200 python -u tools/enc_ser_rates.py | sed "s/^{/{\"streams\": $1, /" >> $OUT/enc_ser.jsonl 2>> $OUT/trace_$1_$2.err || exit 3
  done
done
cat $OUT/enc_ser.jsonl
tail -n 1 $OUT/trace_1_524288.err | cut -c1-700
tail -n 1 $OUT/trace_1_262144.err | cut -c1-700
