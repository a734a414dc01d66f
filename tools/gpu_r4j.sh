#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r4j
timeout -k 10 200 python -u tools/dbg/wavedig_dbg.py > gpurun_out/r4j/wd1.log 2>&1; echo "rc=$?"; cat gpurun_out/r4j/wd1.log | tail -6
XHE_WAVEDIG=0 timeout -k 10 200 python -u tools/dbg/wavedig_dbg.py > gpurun_out/r4j/wd0.log 2>&1; echo "rc=$?"; tail -6 gpurun_out/r4j/wd0.log
