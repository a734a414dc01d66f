#!/bin/bash
# One gpurun call: GPU test suite, default bench line, optional rocprofv3
# passes. Ordinary test failures (pytest exit 1) do not stop the script; a
# crash, abort or time limit of any GPU step does (nothing else runs on the
# GPU after it).
#   tools/gpu_round.sh TAG [step ...]   (default: tests bench)
# steps: tests smoke bench prof lr lrsync lrtrace opstrace configs prodwin
#        rates (RATES_ONLY=add,sum,... RATES_ENV="XHE_X=0 ...": an A/B side)
#        distab (plain vs --dist headline, alternating) proxy (--proxy-world 8 vs 0) cfg4dist pmcops
# Env: PYTEST_ARGS, BENCH_ARGS, RATES_ONLY, RATES_ENV, PMC_ONLY.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-r2}
shift
STEPS=${*:-tests bench}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for s in $STEPS; do
  case $s in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
        ${PYTEST_ARGS} > "$OUT/gpu_tests.log" 2>&1
      rc=$?
      tail -3 "$OUT/gpu_tests.log"
      if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
      ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit $?
      cat "$OUT/smoke.log"
      ;;
    bench)
      timeout -k 10 600 python -u bench.py ${BENCH_ARGS} > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 3; }
      cat "$OUT/bench.json"
      ;;
    prof)
      bash tools/profile_box.sh "$TAG/prof" || exit $?
      ;;
    lr)
      timeout -k 10 600 python -u tools/lr_he_demo.py --epochs 3 --check > "$OUT/lr_demo.json" 2> "$OUT/lr_demo.err" || { tail -20 "$OUT/lr_demo.err"; exit 3; }
      tail -c 1500 "$OUT/lr_demo.json"
      ;;
    lrtrace)
      # rocprofv3 kernel trace of the LR demo (config 1): per-kernel split of a batch
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/lr_trace" -o lr --output-format csv -- \
        python3 -u tools/lr_he_demo.py --epochs 3 --check > "$OUT/lr_demo_prof.json" 2> "$OUT/lr_trace.err" \
        || { tail -20 "$OUT/lr_trace.err"; exit 3; }
      tail -c 600 "$OUT/lr_demo_prof.json"
      ;;
    opstrace)
      # kernel trace of the bench incl. the secondary operations (ops)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/ops_trace" -o ops --output-format csv -- \
        python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/bench_ops_prof.json" 2> "$OUT/ops_trace.err" \
        || { tail -20 "$OUT/ops_trace.err"; exit 3; }
      ;;
    configs)
      bash tools/gpu_configs.sh "$TAG/configs" || exit $?
      ;;
    prodwin)
      # parity at the production fixed-base windows (193-225 GB tables)
      timeout -k 10 900 python -u -m pytest tests/test_gpu_prod_windows.py -v --timeout 600 --timeout-method thread \
        > "$OUT/prodwin.log" 2>&1
      rc=$?
      tail -12 "$OUT/prodwin.log"
      [ $rc -eq 0 ] || exit $rc
      ;;
    rates)
      env $RATES_ENV timeout -k 10 400 python -u tools/rates_r4.py ${RATES_ONLY:+--only $RATES_ONLY} \
        >> "$OUT/rates.jsonl" 2> "$OUT/rates.err" || { tail -5 "$OUT/rates.err"; exit 3; }
      cut -c1-200 "$OUT/rates.jsonl"
      ;;
    lrsync)
      timeout -k 10 300 python -u tools/lr_he_demo.py --epochs 3 --cpu-batches 0 --sync-phases --per-batch \
        --profile-first > "$OUT/lr_sync.json" \
        2> "$OUT/lr_sync.err" || { tail -5 "$OUT/lr_sync.err"; exit 3; }
      tail -c 1500 "$OUT/lr_sync.json"
      ;;
    distab)
      for r in 1 2; do
        for d in "" "--dist"; do
          f="$OUT/headline${d:+_dist}_$r.json"
          timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-ops --no-cpu-baseline $d $BENCH_ARGS > "$f" \
            2> "$f.err" || { tail -5 "$f.err"; exit 3; }
          grep "^{" "$f" | cut -c1-300
        done
      done
      ;;
    proxy)
      # the 8-rank job's gather volume and memory on one GPU (bench.py --proxy-world 8), alternating with the
      # plain RCCL-path run, 20 steps each
      for r in 1 2; do
        for p in 0 8; do
          f="$OUT/proxy${p}_$r.json"
          timeout -k 10 400 python -u bench.py --dist --proxy-world $p --steps 20 --warmup 2 --no-ops \
            --no-cpu-baseline $BENCH_ARGS > "$f" 2> "$f.err" || { tail -5 "$f.err"; exit 3; }
          grep "^{" "$f" | cut -c1-400
        done
      done
      ;;
    cfg4dist)
      timeout -k 10 600 python -u bench.py --key-bits 3072 --n 500000 --gpus 1 --dist --steps 5 --warmup 2 --no-ops \
        --no-cpu-baseline > "$OUT/cfg4_bench_dist.json" 2> "$OUT/cfg4_bench_dist.err" \
        || { tail -20 "$OUT/cfg4_bench_dist.err"; exit 3; }
      cat "$OUT/cfg4_bench_dist.json"
      ;;
    pmcops)
      bash tools/pmc_ops.sh "$TAG/pmc_ops" "${PMC_ONLY:-add,sum,matvec,pub}" || exit $?
      ;;
    *)
      echo "unknown step $s"; exit 2
      ;;
  esac
done
echo "gpu_round $TAG done"
