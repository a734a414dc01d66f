set -e
cd "$GRAFT_REPO_ROOT"
timeout -k 10 60 ./tests/native/_build/mont_selftest > gpurun_out/selftest.log 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "4096 or 3072" > gpurun_out/gpu_tests_4096.log 2>&1
echo ok
