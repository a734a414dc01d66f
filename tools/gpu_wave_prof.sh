# k_dec_wave phase profile (dev builds with XHE_WAVE_PROF=1): cycles per phase over one residue's exponentiation
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for lib in "$@"; do
  echo "== $lib"
  XHE_LIB=$lib XHE_DEC_TPI=64 timeout -k 10 120 python tools/dec_shapes.py 15 2>&1 | grep -v amdgpu.ids | tail -3 || exit 1
done
