cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3g
timeout -k 10 300 python -u -m pytest tests/test_gpu_ndig.py tests/test_gpu_shapes.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r3g/ndig.log 2>&1; rc=$?; tail -3 gpurun_out/r3g/ndig.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/ab_ndig.py > gpurun_out/r3g/ab.jsonl 2> gpurun_out/r3g/ab.err || { tail -5 gpurun_out/r3g/ab.err; exit 3; }
cat gpurun_out/r3g/ab.jsonl
