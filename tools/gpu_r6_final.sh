# round 6: the full GPU suite, smoke and the default bench on the shipped library
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r6final}; mkdir -p $OUT
bash tools/gpu_r6_suite.sh ${1:-r6final} || exit $?
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -n 5 $OUT/bench.err; exit 3; }
tail -c 300 $OUT/bench.json
