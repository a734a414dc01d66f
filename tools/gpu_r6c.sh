cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r6c}; mkdir -p $OUT
timeout -k 10 300 python -u tools/ser_breakdown.py > $OUT/ser.json 2> $OUT/ser.err || { tail -30 $OUT/ser.err; exit 3; }
cat $OUT/ser.json
timeout -k 10 300 python -u tools/rates_r4.py --only pub,add,sum > $OUT/rates.jsonl 2> $OUT/rates.err || { tail -5 $OUT/rates.err; exit 3; }
cut -c1-200 $OUT/rates.jsonl
