# 4-lane Montgomery-digit DJN encryption (3072/4096 bits): parity, then a
# same-box A/B of bench.py against the previous build (xfl_amd/lib/ab_base.so)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3i
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shapes.py tests/test_gpu_codec.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3i/tests.log 2>&1; rc=$?; tail -3 gpurun_out/r3i/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
for kb in 3072 4096; do
  n=500000; [ $kb = 4096 ] && n=262144
  for lib in ab_base.so libxhe.so; do
    XHE_LIB=xfl_amd/lib/$lib timeout -k 10 300 python -u bench.py --key-bits $kb --n $n --steps 3 --warmup 1 --no-ops --no-cpu-baseline > gpurun_out/r3i/bench_${kb}_${lib}.json 2> gpurun_out/r3i/bench_${kb}_${lib}.err || { tail -5 gpurun_out/r3i/bench_${kb}_${lib}.err; exit 3; }
    python -c "import json,sys;r=json.load(open(sys.argv[1]));print(sys.argv[1], r['value'], r['roofline']['kernel_avg_ms'], r['config']['fixed_base_window_bits'], r['parity_sample_ok'])" gpurun_out/r3i/bench_${kb}_${lib}.json
  done
done
timeout -k 10 300 python -u tools/lr_he_demo.py --epochs 3 --check > gpurun_out/r3i/lr_demo.json 2> gpurun_out/r3i/lr.err || { tail -5 gpurun_out/r3i/lr.err; exit 3; }
python -c "import json;r=json.load(open('gpurun_out/r3i/lr_demo.json'));print(r['steady_per_batch_ms'],r['steady_batch_total_ms'],r['checked_bit_exact'])"
