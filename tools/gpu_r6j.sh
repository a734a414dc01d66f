# round 6: k_dec_rns at 4 waves/SIMD (two blocks per CU) and the
# encrypt -> serialize pipeline over a running encryption: parity, the probe,
# the decrypt A/B against the 4-wave build, the LR demo, then the bench
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r6j}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  -k "decrypt" tests/test_gpu_serialize_pipeline.py tests/test_gpu_dropin.py tests/test_gpu_codec.py > $OUT/tests.log 2>&1; rc=$?
tail -n 5 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
XHE_LIB=xfl_amd/lib/probe/libxhe.so timeout -k 10 120 python -u tools/rns_probe.py 15 > $OUT/rns_probe.jsonl 2> $OUT/rns_probe.err || { tail -n 5 $OUT/rns_probe.err; exit 3; }
tail -n 1 $OUT/rns_probe.jsonl
for r in 1 2; do
  XHE_LIB=xfl_amd/lib/ab_v1/libxhe.so timeout -k 10 200 python -u tools/dec_shapes.py 1 15 64 256 512 1024 >> $OUT/dec_v1.jsonl 2>> $OUT/dec.err || exit 3
  timeout -k 10 200 python -u tools/dec_shapes.py 1 15 64 256 512 1024 >> $OUT/dec_v2.jsonl 2>> $OUT/dec.err || exit 3
done
cat $OUT/dec_v1.jsonl $OUT/dec_v2.jsonl
timeout -k 10 300 python -u tools/lr_he_demo.py --epochs 3 --cpu-batches 0 --sync-phases > $OUT/lr_sync.json 2> $OUT/lr_sync.err || { tail -n 5 $OUT/lr_sync.err; exit 3; }
tail -c 400 $OUT/lr_sync.json
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -n 5 $OUT/bench.err; exit 3; }
python - $OUT/bench.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
o = d["ops"]
print(d["value"], {k: o[k] for k in o if k.startswith("dropin_encrypt") or k.startswith("decrypt") or k == "add_per_s"})
PY
