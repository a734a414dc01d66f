cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 120 ./tests/native/_build/pdigit_selftest > gpurun_out/pdigit_selftest.log 2>&1; rc=$?; cat gpurun_out/pdigit_selftest.log; [ $rc -ne 0 ] && exit $rc
AB_TAG=abdec3 bash tools/gpu_ab_dec.sh xfl_amd/lib/ab_pmd3.so xfl_amd/lib/ab_base.so
