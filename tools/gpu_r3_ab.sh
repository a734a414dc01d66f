#!/bin/bash
# round-3 kernel A/B: digit self-test, then tools/gpu_ab.sh on the given libraries
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 120 ./tests/native/_build/pdigit_selftest > gpurun_out/pdigit_selftest.log 2>&1
rc=$?; cat gpurun_out/pdigit_selftest.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_ab.sh "$@"
