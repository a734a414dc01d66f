#!/bin/bash
# Round-4 validation call 3: GPU suite on the in-tree library, LR demo, bench,
# and same-box A/B rates: the in-tree build vs xfl_amd/lib/libxhe_ab.so (the
# same sources without the register-direct word stores) and $XHE_SUM_WORDS=0.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-r4f}
O=gpurun_out/$TAG; mkdir -p $O
bash tools/gpu_round.sh $TAG tests lr || exit $?
R="add,sum,lr,matvec,pub,dec3072"
timeout -k 10 300 python -u tools/rates_r4.py --only $R > $O/rates_new.jsonl 2> $O/rates_new.err || { tail -5 $O/rates_new.err; exit 3; }
XHE_LIB=$PWD/xfl_amd/lib/libxhe_ab.so timeout -k 10 300 python -u tools/rates_r4.py --only $R > $O/rates_ab.jsonl 2> $O/rates_ab.err || { tail -5 $O/rates_ab.err; exit 3; }
XHE_SUM_WORDS=0 timeout -k 10 300 python -u tools/rates_r4.py --only $R > $O/rates_sumrows.jsonl 2> $O/rates_sumrows.err || { tail -5 $O/rates_sumrows.err; exit 3; }
cat $O/rates_new.jsonl $O/rates_ab.jsonl $O/rates_sumrows.jsonl | cut -c1-160
bash tools/gpu_round.sh $TAG bench || exit $?
echo "r4f done"
