# k_dec_wave (one-wave small-batch decrypt) on a 2048-only dev build: parity, then latency per batch size vs the 16-lane shape
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export XHE_LIB=${XHE_LIB:-xfl_amd/lib/dev2048.so}
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "decrypt and 2048" > gpurun_out/wave_par.log 2>&1 || { tail -40 gpurun_out/wave_par.log; exit 1; }
tail -3 gpurun_out/wave_par.log
XHE_DEC_TPI=64 timeout -k 10 120 python tools/dec_shapes.py 1 15 64 256 512 1024 2048 | tee gpurun_out/wave_shapes.log || exit 1
XHE_DEC_TPI=16 timeout -k 10 120 python tools/dec_shapes.py 1 15 64 256 512 1024 2048 | tee -a gpurun_out/wave_shapes.log || exit 1
