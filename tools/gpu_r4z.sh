#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4z; mkdir -p $O
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 3; }
grep "^{" $O/bench.json | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], json.dumps(d['roofline']))"
