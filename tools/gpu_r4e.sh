#!/bin/bash
# Round-4 validation call 2: GPU suite, LR demo (no profiler) + host cProfile,
# same-box A/B rates of the round-4 kernels. Each GPU step has its own limit.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-r4e}
O=gpurun_out/$TAG; mkdir -p $O
bash tools/gpu_round.sh $TAG tests lr || exit $?
timeout -k 10 300 python -u tools/_prof_lr.py > $O/prof_lr.txt 2> $O/prof_lr.err || { tail -5 $O/prof_lr.err; exit 3; }
timeout -k 10 300 python -u tools/rates_r4.py > $O/rates_new.jsonl 2> $O/rates_new.err || { tail -5 $O/rates_new.err; exit 3; }
cat $O/rates_new.jsonl
XHE_NODJN_PMD=0 XHE_DEC_PMDX=0 XHE_NDIG_PUB=0 XHE_MEXP_WAVE=0 XHE_ADD_WAVE=0 timeout -k 10 300 python -u tools/rates_r4.py \
  > $O/rates_old.jsonl 2> $O/rates_old.err || { tail -5 $O/rates_old.err; exit 3; }
cat $O/rates_old.jsonl
echo "r4e done"
