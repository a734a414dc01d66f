#!/bin/bash
# Validation of the shipped build: GPU suite, LR demo, short A/B rates, bench.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-r4m}
O=gpurun_out/$TAG; mkdir -p $O
bash tools/gpu_round.sh $TAG tests lr || exit $?
timeout -k 10 300 python -u tools/rates_r4.py --only add,sum,lr,matvec,pub,nodjn,dec3072 > $O/rates.jsonl 2> $O/rates.err || { tail -5 $O/rates.err; exit 3; }
cut -c1-160 $O/rates.jsonl
bash tools/gpu_round.sh $TAG bench || exit $?
echo "$TAG done"
