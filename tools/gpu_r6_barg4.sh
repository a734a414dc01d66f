# round 6: k_add_barrett with 4 lanes per element (16-column rounds) vs 8 - parity, then same-box A/B
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r6barg4}; mkdir -p $OUT
XHE_LIB=xfl_amd/lib/barg4/libxhe.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_add_barrett.py > $OUT/tests.log 2>&1; rc=$?
tail -n 3 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  timeout -k 10 300 python -u tools/rates_r4.py --only pub,add >> $OUT/g8.jsonl 2>> $OUT/err.log || exit 3
  XHE_LIB=xfl_amd/lib/barg4/libxhe.so timeout -k 10 300 python -u tools/rates_r4.py --only pub,add >> $OUT/g4.jsonl 2>> $OUT/err.log || exit 3
done
grep add_2048 $OUT/g8.jsonl $OUT/g4.jsonl | cut -c1-200
