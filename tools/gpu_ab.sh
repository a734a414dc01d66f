#!/bin/bash
# A/B of development builds (tools/gpu_ab.sh LIB_A LIB_B ...): the 2048-bit
# parity tests on the first library, then bench.py (no ops / baseline) on each.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${AB_TAG:-ab}; mkdir -p $OUT
first=$1
XHE_LIB=$PWD/$first timeout -k 10 600 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_parity.py \
  tests/test_gpu_dropin.py tests/test_gpu_shapes.py -m gpu -k "2048" -q --timeout 300 --timeout-method thread \
  > $OUT/tests.log 2>&1; rc=$?; tail -3 $OUT/tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
for lib in "$@"; do
  tag=$(basename $lib .so)
  XHE_LIB=$PWD/$lib timeout -k 10 300 python bench.py --no-ops --no-cpu-baseline --steps 5 ${BENCH_ARGS} \
    > $OUT/bench_$tag.json 2> $OUT/bench_$tag.err || exit 3
  python -c "import json; r=json.load(open('$OUT/bench_$tag.json')); print('$tag', round(r['value']), round(r['ms_per_step'],3), round(r['roofline']['kernel_avg_ms'],3), round(r['roofline']['frac'],4), r['parity_sample_ok'])"
done
