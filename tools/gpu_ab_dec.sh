#!/bin/bash
# A/B of decrypt / non-DJN kernels (tools/gpu_ab_dec.sh LIB_A LIB_B ...): the
# 2048-bit parity tests on the first library, then tools/dec_rate.py on each.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${AB_TAG:-abdec}; mkdir -p $OUT
XHE_LIB=$PWD/$1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dropin.py \
  tests/test_gpu_codec.py tests/test_gpu_shapes.py -m gpu -k "2048 and not 8192" -q --timeout 300 \
  --timeout-method thread > $OUT/tests.log 2>&1; rc=$?; tail -3 $OUT/tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
for lib in "$@"; do
  XHE_LIB=$PWD/$lib timeout -k 10 300 python tools/dec_rate.py >> $OUT/dec_rate.jsonl 2> $OUT/dec_rate.err || exit 3
  tail -1 $OUT/dec_rate.jsonl
done
