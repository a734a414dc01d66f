#!/bin/bash
# Round-4 counter call: the headline kernel's PMC passes (tools/profile_box.sh)
# and the secondary operations' (tools/pmc_ops.sh), each pass its own run.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-r4d}
mkdir -p gpurun_out/$TAG
bash tools/profile_box.sh "$TAG/prof" || exit $?
bash tools/pmc_ops.sh "$TAG/ops" || exit $?
bash tools/gpu_round.sh "$TAG" lrtrace || exit $?
echo "r4d done"
