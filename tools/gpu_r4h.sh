#!/bin/bash
# Isolate the 3072-bit failure of the in-tree build: pmdx decrypt switched off,
# then each decrypt shape separately (no -x), each under its own time limit.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4h; mkdir -p $O
XHE_DEC_PMDX=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_dropin.py::test_larger_keys_tolerance_ops -k 3072 -v --timeout 120 --timeout-method thread > $O/nopmdx.log 2>&1
echo "nopmdx rc=$?"; grep -E "PASSED|FAILED|Error" $O/nopmdx.log | head
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py::test_decrypt_shapes_bit_exact -k "3072 and (5000 or 30000)" -v --timeout 60 --timeout-method thread > $O/dec.log 2>&1
echo "dec rc=$?"; grep -E "PASSED|FAILED|Error|Timeout" $O/dec.log | head
