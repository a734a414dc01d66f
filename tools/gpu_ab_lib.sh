#!/bin/bash
# Same-box A/B of a development library against the shipped one on tools/rates_r4.py
# (each side its own process, alternating), after the dev library's parity tests.
#   tools/gpu_ab_lib.sh TAG DEV_LIB OPS "PYTEST_FILES" [PMC]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=$1; DEV=$2; OPS=$3; FILES=$4; PMC=$5
O=gpurun_out/$TAG; mkdir -p $O
if [ -n "$FILES" ]; then
  XHE_LIB=$PWD/$DEV timeout -k 10 600 python -u -m pytest $FILES -x -v --timeout 300 --timeout-method thread > $O/tests_dev.log 2>&1
  rc=$?; tail -3 $O/tests_dev.log; [ $rc -eq 0 ] || exit $rc
fi
for r in 1 2; do
  timeout -k 10 300 python -u tools/rates_r4.py --only $OPS >> $O/rates_main.jsonl 2>> $O/rates.err || exit 3
  XHE_LIB=$PWD/$DEV timeout -k 10 300 python -u tools/rates_r4.py --only $OPS >> $O/rates_dev.jsonl 2>> $O/rates.err || exit 3
done
echo main; cut -c1-200 $O/rates_main.jsonl; echo dev; cut -c1-200 $O/rates_dev.jsonl
if [ -n "$PMC" ]; then
  for C in "SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_INSTS_LDS" "SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS" FETCH_SIZE WRITE_SIZE; do
    tag=$(echo "$C" | tr ' ' '_')
    XHE_LIB=$PWD/$DEV timeout -s KILL 300 rocprofv3 --pmc $C --kernel-trace -d "$O/pmc_$tag" -o pmc --output-format csv -- \
      python3 tools/rates_r4.py --only "$OPS" > "$O/pmcrates_$tag.jsonl" 2> "$O/pmc_$tag.err" || { tail -5 "$O/pmc_$tag.err"; exit 3; }
  done
fi
echo "ab $TAG done"
