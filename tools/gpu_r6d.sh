cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r6d}; mkdir -p $OUT
timeout -k 10 120 python -u tools/hostmem_probe.py > $OUT/hostmem.json 2> $OUT/hostmem.err || { tail -30 $OUT/hostmem.err; exit 3; }
cat $OUT/hostmem.json
timeout -k 10 300 python -u tools/ser_breakdown.py > $OUT/ser.json 2> $OUT/ser.err || { tail -30 $OUT/ser.err; exit 3; }
cat $OUT/ser.json
