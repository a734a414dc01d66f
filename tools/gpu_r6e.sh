cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r6e}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_serialize_pipeline.py \
  tests/test_gpu_dropin.py tests/test_gpu_host_pipeline.py tests/test_gpu_parity.py > $OUT/tests.log 2>&1; rc=$?
tail -5 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/ser_breakdown.py > $OUT/ser.json 2> $OUT/ser.err || { tail -30 $OUT/ser.err; exit 3; }
cat $OUT/ser.json
