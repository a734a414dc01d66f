"""Report, per kernel in xhe.hip, VGPRs/scratch and how many scratch
instructions sit inside loops (by the LLVM loop-depth block comments).

    python tools/scratch_report.py   (device-only asm compile for gfx950)
"""
import re
import subprocess
import sys
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = os.path.join(ROOT, "xfl_amd", "csrc", "xhe.hip")
out = "/tmp/xhe_report.s"
subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-S", "--cuda-device-only",
                src, "-o", out], check=True)
s = open(out).read()
rows = []
for m in re.finditer(r"^(_Z\w+):", s, re.M):
    name = m.group(1)
    end = s.find(".Lfunc_end", m.end())
    body = s[m.end():end].split("\n")
    depth = 0
    inloop = outloop = 0
    maxd = 0
    for ln in body:
        b = re.match(r"^\.LBB\d+_\d+:\s*(;.*)?$", ln)
        if b:
            c = b.group(1) or ""
            d = re.search(r"Depth=(\d+)", c)
            depth = int(d.group(1)) if d else 0
            maxd = max(maxd, depth)
        if "scratch_" in ln:
            if depth >= 1:
                inloop += 1
            else:
                outloop += 1
    meta = re.search(r"\.vgpr_count:\s+(\d+)", s[end:end + 4000])
    rows.append((name, inloop, outloop, maxd))
dem = subprocess.run(["c++filt"], input="\n".join(r[0] for r in rows), capture_output=True,
                     text=True).stdout.split("\n")
for r, d in zip(rows, dem):
    if r[1] or r[2] or "-a" in sys.argv:
        print(f"{r[1]:5d} in-loop {r[2]:5d} outside  depth {r[3]}  {d[:110]}")
