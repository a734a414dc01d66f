#!/bin/bash
# k_dec_wave waves per residue (XHE_DEC_NWV 4 / 8 / 16, 2048-only dev builds):
# decrypt parity on each, then latency per batch size, alternating builds.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4o; mkdir -p $O
for v in 8 16; do
  XHE_LIB=$PWD/xfl_amd/lib/dev_nwv$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "decrypt and 2048 and not 30000 and not 20000 and not 5000" -x -q --timeout 120 --timeout-method thread > $O/parity_$v.log 2>&1
  rc=$?; echo "nwv$v parity rc=$rc $(tail -1 $O/parity_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
for r in 1 2; do for v in 4 8 16; do
  XHE_LIB=$PWD/xfl_amd/lib/dev_nwv$v.so XHE_DEC_TPI=64 timeout -k 10 120 python -u tools/dec_shapes.py 1 15 64 256 512 > $O/shapes_${v}_$r.json 2>&1 || exit 3
  echo "nwv$v: $(tail -1 $O/shapes_${v}_$r.json | cut -c1-300)"
done; done
