"""Build the in-tree native library: xfl_amd/lib/libxhe.so (gfx950).

    python -m xfl_amd.build [--force]

hipcc cross-compiles for gfx950 without a GPU, so this runs anywhere the
ROCm toolchain is installed. The .so stays in-tree (not installed) so it
ships with the repository snapshot to the GPU box.
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "lib", "libxhe.so")
SOURCES = [os.path.join(CSRC, f) for f in ("xhe.hip", "xhe_kernels.hpp", "bn_dev.hpp", "hostbn.hpp", "wire.hpp")] + [
    os.path.join(ROOT, "include", "xhe.h")]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("XHE_OFFLOAD_ARCH", "gfx950")


def needs_build():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    return any(os.path.getmtime(s) > t for s in SOURCES)


def build(force=False, verbose=True, out=None, defines=()):
    """Compile libxhe.so. `out`/`defines` build A/B variants of the kernels
    (e.g. defines=["XHE_NPIPE=0"], loaded through $XHE_LIB)."""
    lib = out or LIB
    if not force and out is None and not defines and not needs_build():
        return LIB
    os.makedirs(os.path.dirname(lib), exist_ok=True)
    tmp = lib + ".tmp"
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared"]
    cmd += [f"-D{d}" for d in defines]
    cmd += [os.path.join(CSRC, "xhe.hip"), "-o", tmp]
    if verbose:
        print("[xfl_amd.build]", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(tmp, lib)
    return lib


if __name__ == "__main__":
    args = sys.argv[1:]
    out = args[args.index("--out") + 1] if "--out" in args else None
    defs = [args[i + 1] for i, a in enumerate(args) if a == "-D"]
    build(force="--force" in args, out=out, defines=defs)
