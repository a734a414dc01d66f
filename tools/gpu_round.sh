#!/bin/bash
# One gpurun call: GPU test suite, default bench line, optional rocprofv3
# passes. Ordinary test failures (pytest exit 1) do not stop the script; a
# crash, abort or time limit of any GPU step does (nothing else runs on the
# GPU after it).
#   tools/gpu_round.sh TAG [tests|smoke|bench|prof|lr ...]   (default: tests bench)
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
    *)
      echo "unknown step $s"; exit 2
      ;;
  esac
done
echo "gpu_round $TAG done"
