#!/bin/bash
# Round-4 validation after the store_words rewrite: the multi-lane decrypt
# shapes first (where the per-lane-branch form failed), then tools/gpu_r4f.sh
# (GPU suite, LR demo, A/B rates, bench).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4i; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py::test_decrypt_shapes_bit_exact tests/test_gpu_dropin.py::test_larger_keys_tolerance_ops \
  -k "3072 or 4096" -x -q --timeout 120 --timeout-method thread --tb=line > $O/pmdx.log 2>&1
rc=$?; tail -3 $O/pmdx.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_r4f.sh r4i
