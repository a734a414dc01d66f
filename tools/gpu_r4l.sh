#!/bin/bash
# WaveDig A/B on the LR demo (config 1): whole-wave digit kernels on / off,
# plus a kernel trace with them on.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4l; mkdir -p $O
for v in 1 0 1 0; do
  XHE_WAVEDIG=$v timeout -k 10 300 python -u tools/lr_he_demo.py --epochs 3 --cpu-batches 0 > $O/lr_wd$v.json 2> $O/lr_wd$v.err || { tail -5 $O/lr_wd$v.err; exit 3; }
  python -c "import json;d=json.load(open('$O/lr_wd$v.json'));print('wavedig=$v',{k:round(x,3) for k,x in d['steady_per_batch_ms'].items()},round(d['steady_batch_total_ms'],3))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o lr --output-format csv -- python3 tools/lr_he_demo.py --epochs 2 --cpu-batches 0 > $O/lr_trace.json 2> $O/lr_trace.err || { tail -5 $O/lr_trace.err; exit 3; }
echo "r4l done"
