#!/bin/bash
# Lanes per element of k_djn_pmd for small encrypt batches (XHE_PMD_SPLIT 1/4/16)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4w; mkdir -p $O
for r in 1 2; do for g in 16 4 1; do
  XHE_PMD_SPLIT=$g timeout -k 10 120 python -u tools/dec_shapes.py --enc 15 64 256 1024 > $O/enc_${g}_$r.json 2>&1 || exit 3
  echo "split $g: $(tail -1 $O/enc_${g}_$r.json | cut -c1-260)"
done; done
