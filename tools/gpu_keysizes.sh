# GPU box: Montgomery selftest, the 8192-bit parity tests, then the full GPU
# suite and the per-key-size bench. Each GPU step has its own time limit.
set -e
cd "$GRAFT_REPO_ROOT"
timeout -k 10 60 ./tests/native/_build/mont_selftest > gpurun_out/selftest.log 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "8192" > gpurun_out/gpu_tests_8192.log 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 600 python -u tools/bench_keysizes.py > gpurun_out/keysizes.jsonl 2> gpurun_out/keysizes.err
echo ok
