# round 6: the full GPU suite and smoke on the shipped library
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r6suite}; mkdir -p $OUT
timeout -k 10 1050 python -u -m pytest -m gpu -q --timeout 300 --timeout-method thread tests/ > $OUT/gpu_tests.log 2>&1; rc=$?
tail -n 5 $OUT/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -n 5 $OUT/smoke.log; exit 3; }
tail -n 2 $OUT/smoke.log
