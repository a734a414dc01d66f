#!/bin/bash
# 3072-bit decrypt: kernel trace + VALU-busy pass (tools/pmc_ops.sh with dec3072)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/pmc_ops.sh r4t_dec "dec3072" || exit 3
echo "r4t done"
