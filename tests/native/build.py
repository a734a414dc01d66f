"""Build the device self-test harnesses of tests/native (test infrastructure,
not the product): mont_selftest (Mont<S, W, TPI> products against host big
integers for every limb shape) and pdigit_selftest (base-P digit arithmetic
mod P^2). hipcc cross-compiles for gfx950 without a GPU; the
binaries land in tests/native/_build (git-ignored, shipped to the GPU box with
the tree) and are run by tests/test_gpu_native_selftests.py.

    python tests/native/build.py
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
OUT = os.path.join(HERE, "_build")
CSRC = os.path.join(ROOT, "xfl_amd", "csrc")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
TARGETS = {
    "mont_selftest": ["bn_dev.hpp", "hostbn.hpp"],
    "pdigit_selftest": ["bn_dev.hpp", "hostbn.hpp", "pdigit_dev.hpp"],
}


def _stale(exe, deps):
    if not os.path.exists(exe):
        return True
    t = os.path.getmtime(exe)
    return any(os.path.getmtime(d) > t for d in deps)


def build(verbose=True):
    os.makedirs(OUT, exist_ok=True)
    for name, hdrs in TARGETS.items():
        src = os.path.join(HERE, name + ".hip")
        exe = os.path.join(OUT, name)
        if not _stale(exe, [src] + [os.path.join(CSRC, h) for h in hdrs]):
            continue
        cmd = [HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", src, "-o", exe + ".tmp"]
        if verbose:
            print("[tests/native]", " ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
        os.replace(exe + ".tmp", exe)


if __name__ == "__main__":
    build()
    sys.exit(0)
