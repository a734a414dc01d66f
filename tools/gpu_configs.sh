#!/bin/bash
# GPU box: BASELINE configs 2-5 on one GPU, config 5 as two ranks sharing the
# GPU (gloo; the merge path of the 8-GPU job), and the per-key-size rates.
# Every GPU step has its own time limit; the first failure ends the script.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-configs}
mkdir -p "$OUT"
timeout -k 10 600 python -u tools/bench_configs.py > "$OUT/configs.jsonl" 2> "$OUT/configs.err" || { tail -20 "$OUT/configs.err"; exit 3; }
cat "$OUT/configs.jsonl"
timeout -k 10 400 python -u tools/bench_configs.py --only cfg5 --gpus 2 > "$OUT/cfg5_2ranks.jsonl" 2> "$OUT/cfg5_2ranks.err" || { tail -20 "$OUT/cfg5_2ranks.err"; exit 3; }
cat "$OUT/cfg5_2ranks.jsonl"
timeout -k 10 600 python -u tools/bench_keysizes.py > "$OUT/keysizes.jsonl" 2> "$OUT/keysizes.err" || { tail -20 "$OUT/keysizes.err"; exit 3; }
cat "$OUT/keysizes.jsonl"
