"""Build recipe for the oracle's native pieces (test infrastructure only).

The reference (XFL) ships no native code for this path: its arithmetic is the
third-party gmpy2/GMP, absent as source from /root/reference,
so there is no oracle/_ref build. The CPU baseline C port (gmp_baseline.c,
links the system libgmp.so.10 via dlopen) is built here when present.
"""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))


def build():
    src = os.path.join(HERE, "gmp_baseline.c")
    out = os.path.join(HERE, "_build", "libgmp_baseline.so")
    if not os.path.exists(src):
        return None
    if os.path.exists(out) and os.path.getmtime(out) >= os.path.getmtime(src):
        return out
    os.makedirs(os.path.dirname(out), exist_ok=True)
    subprocess.run(["gcc", "-O2", "-fPIC", "-shared", "-pthread", src, "-o", out, "-ldl"], check=True)
    return out
