#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r4k
timeout -k 10 200 python -u tools/dbg/wavedig_replay.py > gpurun_out/r4k/replay.log 2>&1; echo "rc=$?"; tail -8 gpurun_out/r4k/replay.log
