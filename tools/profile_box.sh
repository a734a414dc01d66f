#!/bin/bash
# Runs on the GPU box (gpurun): kernel-trace stats + PMC passes for the bench
# workload. Every GPU step has its own time limit; stop at the first failure.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-prof}
mkdir -p "$OUT"
N=${N:-1000000}
WIN=${WIN:-23}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
  python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-ops --n "$N" --win "$WIN" > "$OUT/bench_trace.json" 2> "$OUT/trace.err"
for C in FETCH_SIZE WRITE_SIZE "SQ_INSTS_VALU SQ_WAVES" "SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU" \
         "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS"; do
  tag=$(echo "$C" | tr ' ' '_')
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace -d "$OUT/pmc_$tag" -o pmc --output-format csv -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-ops --n "$N" --win "$WIN" > "$OUT/bench_$tag.json" 2> "$OUT/pmc_$tag.err"
done
echo done
