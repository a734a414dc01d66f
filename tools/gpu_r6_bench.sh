# round 6: the default bench on the shipped library
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r6bench}; mkdir -p $OUT
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -n 5 $OUT/bench.err; exit 3; }
tail -c 600 $OUT/bench.json
