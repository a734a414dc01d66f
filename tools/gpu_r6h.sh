# round 6: the RNS decrypt's crossover against the 16-lane shape, then the default bench
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r6h}; mkdir -p $OUT
XHE_LIB=xfl_amd/lib/probe/libxhe.so timeout -k 10 120 python -u tools/rns_probe.py 15 > $OUT/rns_probe.jsonl 2> $OUT/rns_probe.err || { tail -5 $OUT/rns_probe.err; exit 3; }
cat $OUT/rns_probe.jsonl
XHE_DEC_TPI=64 timeout -k 10 200 python -u tools/dec_shapes.py 512 768 1024 1536 2048 3072 > $OUT/dec_rns64.jsonl 2>> $OUT/dec.err || exit 3
XHE_DEC_TPI=16 timeout -k 10 200 python -u tools/dec_shapes.py 512 768 1024 1536 2048 3072 > $OUT/dec_row16.jsonl 2>> $OUT/dec.err || exit 3
cat $OUT/dec_rns64.jsonl $OUT/dec_row16.jsonl
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 3; }
tail -c 3000 $OUT/bench.json
