#!/bin/bash
# Same-box A/B of one environment switch of a library: parity tests under every
# value, then a timing command alternated over the values (two rounds).
#   [PYK="-k expression"] tools/gpu_env_ab.sh TAG LIB VAR "V1 V2 ..." "PYTEST_FILES" TIMING_CMD...
# e.g. PYK="decrypt and not 3072" tools/gpu_env_ab.sh w1 xfl_amd/lib/dev2048.so XHE_DEC_W1 "0 1 2" \
#        tests/test_gpu_parity.py python -u tools/dec_shapes.py 1 15 64 256 512
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=$1; LIB=$2; VAR=$3; VALS=$4; PYT=$5; shift 5
O=gpurun_out/$TAG; mkdir -p $O
export XHE_LIB=$PWD/$LIB
if [ -n "$PYT" ]; then
  for v in $VALS; do
    env $VAR=$v timeout -k 10 600 python -u -m pytest $PYT ${PYK:+-k "$PYK"} -x -v --timeout 300 --timeout-method thread > $O/tests_$v.log 2>&1
    rc=$?; echo "$VAR=$v: $(tail -1 $O/tests_$v.log)"; [ $rc -eq 0 ] || exit $rc
  done
fi
for r in 1 2; do
  for v in $VALS; do
    env $VAR=$v timeout -k 10 300 "$@" > $O/t_$v.$r.json 2>> $O/timing.err || exit 3
    echo "$VAR=$v round $r: $(cut -c1-400 $O/t_$v.$r.json)"
  done
done
echo "env ab $TAG done"
