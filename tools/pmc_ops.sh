#!/bin/bash
# GPU box: rocprofv3 counter passes over tools/rates_r4.py (the secondary
# operations: add, sum/histogram, mat-vec, public DJN / non-DJN encryption,
# 3072/4096 decrypt), one pass per counter group (rocprofv3 does not split
# passes), each under its own kill timeout. Summaries: tools/pmc_traffic.py
# per kernel.
#   tools/pmc_ops.sh TAG [OPS]     (OPS: rates_r4.py --only list)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-pmc_ops}
OPS=${2:-pub,add,sum,pubnodjn,matvec}
mkdir -p "$OUT"
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
  python3 tools/rates_r4.py --only "$OPS" > "$OUT/rates_trace.jsonl" 2> "$OUT/trace.err" || { tail -5 "$OUT/trace.err"; exit 3; }
for C in "SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_INSTS_LDS" "SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS" \
         FETCH_SIZE WRITE_SIZE; do
  tag=$(echo "$C" | tr ' ' '_')
  timeout -s KILL 300 rocprofv3 --pmc $C --kernel-trace -d "$OUT/pmc_$tag" -o pmc --output-format csv -- \
    python3 tools/rates_r4.py --only "$OPS" > "$OUT/rates_$tag.jsonl" 2> "$OUT/pmc_$tag.err" || { tail -5 "$OUT/pmc_$tag.err"; exit 3; }
done
echo "pmc_ops $OUT done"
