#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r4u
timeout -k 10 600 python -u -m pytest tests/test_gpu_invert.py -v --timeout 300 --timeout-method thread > gpurun_out/r4u/invert.log 2>&1
rc=$?; tail -8 gpurun_out/r4u/invert.log; exit $rc
