# A/B of k_dec_wave builds (2048-only dev libs): decrypt parity on each, then latency per batch size, alternating
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/abwave; mkdir -p $OUT
for lib in "$@"; do
  XHE_LIB=xfl_amd/lib/$lib timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "decrypt and 2048" > $OUT/par_$lib.log 2>&1 || { tail -20 $OUT/par_$lib.log; exit 1; }
  tail -1 $OUT/par_$lib.log
done
for rep in 1 2; do for lib in "$@"; do
  echo -n "$lib " | tee -a $OUT/ab.txt
  XHE_LIB=xfl_amd/lib/$lib XHE_DEC_TPI=64 timeout -k 10 120 python tools/dec_shapes.py 1 15 64 256 512 2>/dev/null | tee -a $OUT/ab.txt || exit 1
done; done
