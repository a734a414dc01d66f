"""Build the in-tree native library: xfl_amd/lib/libxhe.so (gfx950).

    python -m xfl_amd.build [--force] [--out PATH] [-D NAME[=V] ...]

Two translation units, compiled in parallel into xfl_amd/lib/obj/ and linked
into one shared library:
  xhe.hip       device kernels + the kernel entry points   (hipcc, gfx950)
  wire_abi.cpp  host-only entry points: wire codec, errors (host compiler)
so a codec change rebuilds in seconds and only kernel changes pay for the
device compile. hipcc cross-compiles for gfx950 without a GPU, so this runs
anywhere the ROCm toolchain is installed. The .so stays in-tree (not
installed) so it ships with the repository snapshot to the GPU box.
-D XHE_ONLY_2048 gives a development build with the 2048-bit shapes only
(for kernel A/B runs through $XHE_LIB).
"""
import concurrent.futures
import hashlib
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "lib", "libxhe.so")
OBJ = os.path.join(HERE, "lib", "obj")
HEADER = os.path.join(ROOT, "include", "xhe.h")
DEVICE_DEPS = [os.path.join(CSRC, f) for f in ("xhe.hip", "xhe_kernels.hpp", "bn_dev.hpp", "pdigit_dev.hpp", "dec_wave.hpp", "barrett_dev.hpp", "rns_dev.hpp", "hostbn.hpp",
                                               "abi_common.hpp")] + [HEADER]
HOST_DEPS = [os.path.join(CSRC, f) for f in ("wire_abi.cpp", "wire.hpp", "abi_common.hpp")] + [HEADER]
SOURCES = sorted(set(DEVICE_DEPS + HOST_DEPS))
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CXX = os.environ.get("CXX", "g++")
ARCH = os.environ.get("XHE_OFFLOAD_ARCH", "gfx950")


# warnings that mark undefined behaviour in the kernels are errors (a 32-bit
# shift by 56 once silently dropped a term of WaveDig's top limb)
WERROR = ["-Werror=shift-count-overflow", "-Werror=shift-count-negative"]


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def needs_build():
    return _stale(LIB, SOURCES)


def _run(cmd, verbose):
    if verbose:
        print("[xfl_amd.build]", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)


def build(force=False, verbose=True, out=None, defines=()):
    """Compile libxhe.so. `out`/`defines` build A/B variants of the kernels
    (e.g. defines=["XHE_ONLY_2048"], loaded through $XHE_LIB)."""
    lib = out or LIB
    if not force and out is None and not defines and not needs_build():
        return LIB
    os.makedirs(OBJ, exist_ok=True)
    os.makedirs(os.path.dirname(lib), exist_ok=True)
    tag = hashlib.sha1(" ".join(sorted(defines)).encode()).hexdigest()[:8] if defines else "default"
    dev_obj = os.path.join(OBJ, f"xhe.{tag}.o")
    host_obj = os.path.join(OBJ, "wire_abi.o")
    dflags = [f"-D{d}" for d in defines]
    jobs = []
    if force or _stale(dev_obj, DEVICE_DEPS):
        jobs.append([HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", *WERROR, *dflags, "-c",
                     os.path.join(CSRC, "xhe.hip"), "-o", dev_obj + ".tmp"])
    if force or _stale(host_obj, HOST_DEPS):
        jobs.append([CXX, "-O3", "-std=c++17", "-fPIC", "-pthread", "-c", os.path.join(CSRC, "wire_abi.cpp"),
                     "-o", host_obj + ".tmp"])
    with concurrent.futures.ThreadPoolExecutor(max_workers=2) as ex:
        for f in [ex.submit(_run, j, verbose) for j in jobs]:
            f.result()
    for j in jobs:
        os.replace(j[-1], j[-1][:-4])
    tmp = lib + ".tmp"
    _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-pthread", dev_obj, host_obj, "-o", tmp], verbose)
    os.replace(tmp, lib)
    return lib


if __name__ == "__main__":
    args = sys.argv[1:]
    out = args[args.index("--out") + 1] if "--out" in args else None
    defs = [args[i + 1] for i, a in enumerate(args) if a == "-D"]
    build(force="--force" in args, out=out, defines=defs)
