# 3072-bit k_djn_pmdx: 2 lanes of 30 limbs (ab_3072_t2.so) vs 4 lanes of 15 (libxhe.so), same box
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3j
XHE_LIB=xfl_amd/lib/ab_3072_t2.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k 3072 -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r3j/tests.log 2>&1; rc=$?; tail -2 gpurun_out/r3j/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
for lib in libxhe.so ab_3072_t2.so libxhe.so ab_3072_t2.so; do
  XHE_LIB=xfl_amd/lib/$lib timeout -k 10 300 python -u bench.py --key-bits 3072 --n 500000 --steps 3 --warmup 1 --no-ops --no-cpu-baseline > gpurun_out/r3j/b.json 2> gpurun_out/r3j/b.err || { tail -5 gpurun_out/r3j/b.err; exit 3; }
  python -c "import json,sys;r=json.load(open('gpurun_out/r3j/b.json'));print(sys.argv[1], r['value'], r['roofline']['kernel_avg_ms'])" $lib | tee -a gpurun_out/r3j/ab.txt
done
