# round 6: k_dec_rns on 6 waves (split extension sums, Shoup constants) -
# parity, the cycle probe, then the same-box A/B against the 4-wave build
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r6i}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  -k "decrypt" > $OUT/tests_dec.log 2>&1; rc=$?
tail -n 5 $OUT/tests_dec.log
[ $rc -eq 0 ] || exit $rc
XHE_LIB=xfl_amd/lib/probe/libxhe.so timeout -k 10 120 python -u tools/rns_probe.py 15 > $OUT/rns_probe.jsonl 2> $OUT/rns_probe.err || { tail -n 5 $OUT/rns_probe.err; exit 3; }
cat $OUT/rns_probe.jsonl
for r in 1 2; do
  XHE_LIB=xfl_amd/lib/ab_v1/libxhe.so timeout -k 10 200 python -u tools/dec_shapes.py 1 15 64 256 512 1024 >> $OUT/dec_v1.jsonl 2>> $OUT/dec.err || exit 3
  timeout -k 10 200 python -u tools/dec_shapes.py 1 15 64 256 512 1024 >> $OUT/dec_v2.jsonl 2>> $OUT/dec.err || exit 3
done
cat $OUT/dec_v1.jsonl $OUT/dec_v2.jsonl
timeout -k 10 300 python -u tools/lr_he_demo.py --epochs 3 --cpu-batches 0 --sync-phases > $OUT/lr_sync.json 2> $OUT/lr_sync.err || { tail -n 5 $OUT/lr_sync.err; exit 3; }
tail -c 700 $OUT/lr_sync.json
