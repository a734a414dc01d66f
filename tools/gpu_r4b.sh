cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4b; mkdir -p $O
export XHE_LIB=$PWD/xfl_amd/lib/libxhe_dev1.so
timeout -k 10 700 python -u -m pytest tests/test_gpu_shapes.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/rates_r4.py --only nodjn,dec3072,dec4096 > $O/rates_new.jsonl 2> $O/rates_new.err || { tail -5 $O/rates_new.err; exit 3; }
cat $O/rates_new.jsonl
XHE_NODJN_PMD=0 XHE_DEC_PMDX=0 timeout -k 10 300 python -u tools/rates_r4.py --only nodjn,dec3072,dec4096 > $O/rates_old.jsonl 2> $O/rates_old.err || { tail -5 $O/rates_old.err; exit 3; }
cat $O/rates_old.jsonl
