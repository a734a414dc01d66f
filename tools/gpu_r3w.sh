# Round-3 evidence after k_dec_wave: GPU suite, smoke, default bench, LR demo,
# then the decrypt latency per batch size (auto shapes vs the 16-lane shape)
# and a kernel trace of the small-batch decrypt
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_round.sh r3w ${STEPS:-tests smoke bench lr} || exit $?
OUT=gpurun_out/r3w/wave
mkdir -p $OUT
timeout -k 10 180 python3 tools/dec_shapes.py 1 15 64 256 512 1024 2048 > $OUT/dec_shapes_auto.json || exit 3
XHE_DEC_TPI=16 timeout -k 10 180 python3 tools/dec_shapes.py 1 15 64 256 512 1024 2048 > $OUT/dec_shapes_16.json || exit 3
cat $OUT/dec_shapes_auto.json $OUT/dec_shapes_16.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
  python3 tools/dec_shapes.py 15 64 > $OUT/dec_shapes_traced.json 2> $OUT/trace.err || { tail -5 $OUT/trace.err; exit 3; }
echo done
