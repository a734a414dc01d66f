#!/bin/bash
# Same-box A/B of a development library against the shipped one by rocprofv3
# kernel statistics of one command (each side its own process, alternating,
# two rounds), after the dev library's parity tests.
#   [PYK="-k expression"] tools/gpu_trace_ab.sh TAG DEV_LIB "PYTEST_FILES" PROGRAM ARGS...
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=$1; DEV=$2; PYT=$3; shift 3
O=gpurun_out/$TAG; mkdir -p $O
if [ -n "$PYT" ]; then
  XHE_LIB=$PWD/$DEV timeout -k 10 900 python -u -m pytest $PYT -m gpu ${PYK:+-k "$PYK"} -x -v --timeout 300 \
    --timeout-method thread > $O/tests_dev.log 2>&1
  rc=$?; echo "dev tests: $(tail -1 $O/tests_dev.log)"; [ $rc -eq 0 ] || exit $rc
fi
for r in 1 2; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/main$r -o run --output-format csv -- "$@" \
    > $O/main$r.out 2> $O/main$r.err || exit 3
  XHE_LIB=$PWD/$DEV timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/dev$r -o run --output-format csv -- "$@" \
    > $O/dev$r.out 2> $O/dev$r.err || exit 3
done
for f in $O/main1 $O/dev1 $O/main2 $O/dev2; do
  echo "$f: $(python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$f/run_kernel_stats.csv')))
print('; '.join(r['Name'].split('(')[0].split('<')[0][-22:]+' '+str(round(float(r['AverageNs'])/1e3,1))+'us' for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:6]))
")"
done
echo "trace ab $TAG done"
