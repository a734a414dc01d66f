"""Per-kernel register / LDS / scratch use of the built library (the gfx950
code object inside xfl_amd/lib/libxhe.so), from the code object's metadata
notes - spills show up here without a GPU.

    python tools/kernel_resources.py [name-substring ...]
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def kernels(lib=os.path.join(ROOT, "xfl_amd", "lib", "libxhe.so")):
    with tempfile.TemporaryDirectory() as d:
        fat, co = os.path.join(d, "fat.bin"), os.path.join(d, "x.co")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", lib, os.path.join(d, "junk")],
                       check=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
        notes = subprocess.run([f"{LLVM}/llvm-readobj", "--notes", co], check=True, capture_output=True,
                               text=True).stdout
    out = []
    for b in notes.split("- .agpr_count")[1:]:
        def g(k):
            m = re.search(r"\." + k + r":\s+(\S+)", b)
            return m.group(1) if m else None
        name = g("name")
        demangled = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
        out.append({"kernel": demangled, "vgpr": g("vgpr_count"), "vgpr_spill": g("vgpr_spill_count"),
                    "sgpr_spill": g("sgpr_spill_count"), "lds": g("group_segment_fixed_size"),
                    "scratch": g("private_segment_fixed_size")})
    return out


if __name__ == "__main__":
    pats = sys.argv[1:]
    for k in kernels():
        if not pats or any(p in k["kernel"] for p in pats):
            print(f"{k['kernel'][:90]:90s} vgpr {k['vgpr']:>4} spill {k['vgpr_spill']:>4} sgpr_spill "
                  f"{k['sgpr_spill']:>3} lds {k['lds']:>6} scratch {k['scratch']:>5}")
