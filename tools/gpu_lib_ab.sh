#!/bin/bash
# Same-box A/B of a development library against the shipped one on any timing
# command (each side its own process, alternating, two rounds), after the dev
# library's parity tests.
#   [PYK="-k expression"] tools/gpu_lib_ab.sh TAG DEV_LIB "PYTEST_FILES" TIMING_CMD...
# e.g. PYK=8192 tools/gpu_lib_ab.sh ks8 xfl_amd/lib/dev8192.so tests \
#        python -u tools/bench_keysizes.py --bits 8192
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=$1; DEV=$2; PYT=$3; shift 3
O=gpurun_out/$TAG; mkdir -p $O
if [ -n "$PYT" ]; then
  XHE_LIB=$PWD/$DEV timeout -k 10 900 python -u -m pytest $PYT -m gpu ${PYK:+-k "$PYK"} -x -v --timeout 300 \
    --timeout-method thread > $O/tests_dev.log 2>&1
  rc=$?; echo "dev tests: $(tail -1 $O/tests_dev.log)"; [ $rc -eq 0 ] || exit $rc
fi
for r in 1 2; do
  timeout -k 10 400 "$@" > $O/main.$r.json 2>> $O/timing.err || exit 3
  echo "main round $r: $(cut -c1-400 $O/main.$r.json)"
  XHE_LIB=$PWD/$DEV timeout -k 10 400 "$@" > $O/dev.$r.json 2>> $O/timing.err || exit 3
  echo "dev round $r: $(cut -c1-400 $O/dev.$r.json)"
done
echo "lib ab $TAG done"
