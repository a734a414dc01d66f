# round 6: serialize with device bit lengths behind the pieces - tests, A/B, bench
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r6t}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_serialize_pipeline.py \
  tests/test_gpu_resident.py tests/test_gpu_dropin.py tests/test_gpu_codec.py > $OUT/tests.log 2>&1; rc=$?
tail -n 3 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 200 python -u tools/enc_ser_rates.py >> $OUT/enc_ser.jsonl 2>> $OUT/err.log || exit 3
done
cat $OUT/enc_ser.jsonl
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -n 5 $OUT/bench.err; exit 3; }
python - $OUT/bench.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
o = d["ops"]
print(d["value"], {k: o[k] for k in o if k.startswith("dropin_encrypt") or k.startswith("dropin_serialize")})
PY
