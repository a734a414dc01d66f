cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3e
timeout -k 10 500 python -u -m pytest tests/test_gpu_shapes.py tests/test_gpu_parity.py tests/test_gpu_resident.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r3e/tests.log 2>&1; rc=$?; tail -3 gpurun_out/r3e/tests.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-ops > gpurun_out/r3e/bench.json 2> gpurun_out/r3e/bench.err || exit 3
timeout -k 10 300 python -u tools/lr_he_demo.py --epochs 3 --check > gpurun_out/r3e/lr_demo.json 2> gpurun_out/r3e/lr.err; echo lr rc=$?
python -c "import json;r=json.load(open('gpurun_out/r3e/bench.json'));print(r['value'],r['roofline']['kernel_avg_ms']);r=json.load(open('gpurun_out/r3e/lr_demo.json'));print(r['steady_per_batch_ms'],r['steady_batch_total_ms'])"
