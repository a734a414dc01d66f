cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r6a; mkdir -p $OUT
timeout -k 10 600 python -u tools/groupby_rate.py --profile > $OUT/groupby.json 2> $OUT/groupby.err || { tail -30 $OUT/groupby.err; exit 3; }
cat $OUT/groupby.json
timeout -k 10 300 python -u -m pytest tests/test_gpu_full_configs.py -v --timeout 240 --timeout-method thread -s > $OUT/full_configs.log 2>&1; rc=$?
tail -15 $OUT/full_configs.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --deselect tests/test_gpu_full_configs.py > $OUT/gpu_tests.log 2>&1; rc=$?
tail -5 $OUT/gpu_tests.log
exit $rc
