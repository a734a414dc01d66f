# round 6: async small uploads - the drop-in / resident / LR tests, then the LR demo
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r6n}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_dropin.py \
  tests/test_gpu_resident.py tests/test_gpu_lr_demo.py tests/test_gpu_matvec.py tests/test_gpu_invert.py > $OUT/tests.log 2>&1; rc=$?
tail -n 3 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/lr_he_demo.py --epochs 3 --cpu-batches 0 --sync-phases > $OUT/lr_sync.json 2> $OUT/lr_sync.err || { tail -n 5 $OUT/lr_sync.err; exit 3; }
tail -c 500 $OUT/lr_sync.json
