cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r2split; mkdir -p $OUT
export XHE_LIB=$PWD/xfl_amd/lib/libxhe_dev.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_shapes.py tests/test_gpu_parity.py tests/test_gpu_codec.py -m gpu -k "2048 or both_shapes" -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?; tail -3 $OUT/tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
for w in 23s 23 23s; do
  timeout -k 10 300 python bench.py --no-ops --no-cpu-baseline --steps 5 --win $w > $OUT/bench_$w.json 2> $OUT/bench_$w.err || exit 3
  python -c "import json; r=json.load(open('$OUT/bench_$w.json')); print('$w', round(r['value']), round(r['ms_per_step'],3), round(r['roofline']['kernel_avg_ms'],3), round(r['roofline']['frac'],4), r['parity_sample_ok'], r['key_setup_s'])"
done
