#!/bin/bash
# The plain-aligned add test, an LR kernel trace, then the BASELINE configs
# (tools/gpu_r4g.sh: configs 2-5, cfg5 on 2 ranks, key sizes, cfg4 over RCCL).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4n; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_dropin.py -k "plain_aligned or binary" -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/lrtrace -o lr --output-format csv -- python3 tools/lr_he_demo.py --epochs 2 --cpu-batches 0 > $O/lr_trace.json 2> $O/lr_trace.err || { tail -5 $O/lr_trace.err; exit 3; }
bash tools/gpu_r4g.sh r4n
