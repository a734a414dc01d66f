# round 6: groupby after the async segprod + adaptive chunks, serialize breakdown, targeted tests
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r6b}; mkdir -p $OUT
timeout -k 10 600 python -u tools/groupby_rate.py --profile > $OUT/groupby.json 2> $OUT/groupby.err || { tail -30 $OUT/groupby.err; exit 3; }
cat $OUT/groupby.json
timeout -k 10 300 python -u tools/ser_breakdown.py > $OUT/ser.json 2> $OUT/ser.err || { tail -30 $OUT/ser.err; exit 3; }
cat $OUT/ser.json
timeout -k 10 300 python -u tools/rates_r4.py --only add,sum > $OUT/rates.jsonl 2> $OUT/rates.err || { tail -5 $OUT/rates.err; exit 3; }
cut -c1-300 $OUT/rates.jsonl
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_full_configs.py \
  tests/test_gpu_add_barrett.py tests/test_gpu_dropin.py tests/test_gpu_shapes.py tests/test_gpu_matvec.py \
  tests/test_gpu_lr_demo.py tests/test_gpu_shard.py tests/test_gpu_resident.py tests/test_gpu_rccl.py tests/test_gpu_gather.py \
  > $OUT/tests.log 2>&1; rc=$?
tail -5 $OUT/tests.log
exit $rc
