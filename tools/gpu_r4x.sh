#!/bin/bash
# Final full GPU suite on the round's last tree.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_round.sh r4x tests || exit $?
echo "r4x done"
