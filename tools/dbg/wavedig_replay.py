"""Replay the failing WaveDig operands (tools/dbg/bad_p.json) through the
probe and dump the product's columns (debug tool)."""
import json, os, subprocess, sys
import numpy as np
sys.path.insert(0, os.getcwd())
from tests.conftest import hx, load_fixture
W, K = 28, 37
MASK, R = (1 << W) - 1, 1 << (W * K)
limbs = lambda x: [(x >> (W * i)) & MASK for i in range(K)]
def tol(v):
    l = limbs(v % R); l[-1] += (v >> (W * K)) << W; return l
g = load_fixture("paillier_2048_djn.json")
P = hx(g["key"]["p"]); Pp = (-pow(P, -1, R)) % R; E = (1 - R) % P
topc = [(MASK + x) & 0xFFFFFFFF for x in limbs(E)]
bad = json.load(open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/r4k/bad_p.json"))
ops = [tuple(int(b[k], 16) for k in "acef") for b in bad]
buf = np.array(limbs(P) + limbs(Pp) + topc + [x for o in ops for v in o for x in tol(v)], np.uint32)
os.makedirs("gpurun_out/r4k", exist_ok=True)
buf.tofile("gpurun_out/r4k/rin.bin")
r = subprocess.run(["tools/dbg/wavedig_probe", "gpurun_out/r4k/rin.bin", "gpurun_out/r4k/rout.bin", str(len(ops)),
                    "gpurun_out/r4k/rcols.bin"], capture_output=True, text=True, timeout=60)
print(r.returncode, r.stdout, r.stderr[-300:])
cols = np.fromfile("gpurun_out/r4k/rcols.bin", np.uint64).reshape(len(ops), 2, 3 + 2 * K)
for i in range(len(ops)):
    print(i, "col2[G+69..G+73]", [hex(int(x)) for x in cols[i, 1, 3 + 69:3 + 74]], "guards", [hex(int(x)) for x in cols[i, 1, :3]])
