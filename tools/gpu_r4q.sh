#!/bin/bash
# LR demo per-phase latency (device synchronised at each phase end) and a
# host profile of the steady epochs.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4q; mkdir -p $O
timeout -k 10 300 python -u tools/lr_he_demo.py --epochs 3 --cpu-batches 0 --sync-phases > $O/lr_sync.json 2> $O/lr_sync.err || exit 3
python -c "import json;d=json.load(open('$O/lr_sync.json'));print({k:round(v,3) for k,v in d['steady_per_batch_ms'].items()}, d['steady_batch_total_ms'])"
timeout -k 10 300 python -u tools/_prof_lr.py > $O/prof.txt 2>&1 || exit 3
head -60 $O/prof.txt
