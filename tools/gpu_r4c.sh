#!/bin/bash
# Round-4 validation call: GPU suite, bench, LR trace, same-box A/B of the
# kernels moved to digits this round. Each GPU step has its own time limit;
# a crash/abort/time limit ends the script (test failures do not).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-r4c}
O=gpurun_out/$TAG; mkdir -p $O
bash tools/gpu_round.sh $TAG tests bench lrtrace || exit $?
timeout -k 10 300 python -u tools/rates_r4.py > $O/rates_new.jsonl 2> $O/rates_new.err || { tail -5 $O/rates_new.err; exit 3; }
cat $O/rates_new.jsonl
XHE_NODJN_PMD=0 XHE_DEC_PMDX=0 XHE_NDIG_PUB=0 XHE_MEXP_WAVE=0 timeout -k 10 300 python -u tools/rates_r4.py \
  --only nodjn,pub,dec3072,dec4096,matvec > $O/rates_old.jsonl 2> $O/rates_old.err || { tail -5 $O/rates_old.err; exit 3; }
cat $O/rates_old.jsonl
echo "r4c done"
