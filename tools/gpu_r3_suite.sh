set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./tests/native/_build/pdigit_selftest > gpurun_out/pdigit_selftest.log 2>&1; echo "pdigit rc=$?" >> gpurun_out/pdigit_selftest.log
cat gpurun_out/pdigit_selftest.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -15 gpurun_out/gpu_tests.log
exit $rc
