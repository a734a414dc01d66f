# round 6: encryption launches on two streams + the serialize pipeline over them
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r6k}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_serialize_pipeline.py \
  tests/test_gpu_dropin.py tests/test_gpu_resident.py > $OUT/tests.log 2>&1; rc=$?
tail -n 5 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -n 5 $OUT/bench.err; exit 3; }
python - $OUT/bench.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
o = d["ops"]
print(d["value"], {k: o[k] for k in o if k.startswith("dropin_encrypt") or k.startswith("decrypt") or k == "add_per_s"})
PY
