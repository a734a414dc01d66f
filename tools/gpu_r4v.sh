#!/bin/bash
# After the last host-side changes: drop-in + LR tests, the LR demo, smoke().
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4v; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_dropin.py tests/test_gpu_lr_demo.py tests/test_gpu_resident.py -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/lr_he_demo.py --epochs 3 --check --cpu-batches 0 > $O/lr_demo.json 2> $O/lr_demo.err || exit 3
python -c "import json;d=json.load(open('$O/lr_demo.json'));print({k:round(v,3) for k,v in d['steady_per_batch_ms'].items()}, d['steady_batch_total_ms'], d['checked_bit_exact'])"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1; rc=$?; tail -2 $O/smoke.log; exit $rc
