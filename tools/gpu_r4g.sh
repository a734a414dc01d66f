#!/bin/bash
# Round-4 configs call: BASELINE configs 2-5 (tools/bench_configs.py, config 5
# also as 2 ranks), every key size (tools/bench_keysizes.py), and config 4's
# bench line through the RCCL path at world 1 (bench.py --dist).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-r4g}
O=gpurun_out/$TAG; mkdir -p $O
bash tools/gpu_configs.sh "$TAG/configs" || exit $?
timeout -k 10 600 python -u bench.py --key-bits 3072 --n 500000 --gpus 1 --dist --steps 5 --warmup 2 --no-ops \
  --no-cpu-baseline > $O/cfg4_bench_dist.json 2> $O/cfg4_bench_dist.err || { tail -20 $O/cfg4_bench_dist.err; exit 3; }
cat $O/cfg4_bench_dist.json
echo "r4g done"
