cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3f
timeout -k 10 300 python -u -m pytest tests/test_gpu_ndig.py -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/r3f/ndig.log 2>&1; rc=$?; tail -8 gpurun_out/r3f/ndig.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/ab_ndig.py > gpurun_out/r3f/ab.jsonl 2> gpurun_out/r3f/ab.err || { tail -5 gpurun_out/r3f/ab.err; exit 3; }
cat gpurun_out/r3f/ab.jsonl
if [ $rc -ne 0 ]; then exit 1; fi
timeout -k 10 600 python -u -m pytest tests/test_gpu_shapes.py tests/test_gpu_parity.py tests/test_gpu_dropin.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r3f/tests.log 2>&1; tail -3 gpurun_out/r3f/tests.log
