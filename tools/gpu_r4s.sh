#!/bin/bash
# Final-build profiles: headline kernel trace + PMC passes (tools/profile_box.sh)
# and the mod-n^2 operations' PMC passes (tools/pmc_ops.sh).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/profile_box.sh r4s_head || exit 3
bash tools/pmc_ops.sh r4s_ops "add,sum,matvec,pub" || exit 3
echo "r4s done"
