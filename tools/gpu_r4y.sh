#!/bin/bash
# Headline through the RCCL path at world 1 vs plain, same box, alternating.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4y; mkdir -p $O
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-ops --no-cpu-baseline > $O/plain_$r.json 2> $O/plain_$r.err || exit 3
  timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-ops --no-cpu-baseline --dist > $O/dist_$r.json 2> $O/dist_$r.err || exit 3
  for f in plain_$r dist_$r; do grep "^{" $O/$f.json | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('$f', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],2), 'ms/step', d['config']['parallelism'], round(d['roofline']['kernel_avg_ms'],2))"; done
done
