"""Drive tests/native/wavedig_probe.hip (built as tools/dbg/wavedig_probe):
random digit products mod P^2 for the fixture's p and q, each result checked
as a residue; failing operands saved for the limb-level model. Debug tool."""
import json, os, random, subprocess, sys
import numpy as np
sys.path.insert(0, os.getcwd())
from tests.conftest import hx, load_fixture

W, K = 28, 37
MASK, R = (1 << W) - 1, 1 << (W * K)
limbs = lambda x: [(x >> (W * i)) & MASK for i in range(K)]
val = lambda l: sum(int(v) << (W * i) for i, v in enumerate(l))
g = load_fixture("paillier_2048_djn.json")
n = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
os.makedirs("gpurun_out/r4k", exist_ok=True)
rng = random.Random(11)
for name in ("p", "q"):
    P = hx(g["key"][name]); P2 = P * P
    Pp = (-pow(P, -1, R)) % R
    E = (1 - R) % P
    topc = [(MASK + x) & 0xFFFFFFFF for x in limbs(E)]
    ops = []
    for i in range(n):
        a, c, e, f = (rng.randrange(P) for _ in range(4))
        if i % 4 == 1: c = R + rng.randrange(4 * P)          # c' range of a product
        if i % 4 == 2: a = P + rng.randrange(2 * P * P // R + 1) if 2 * P * P // R else a
        ops.append((a, c, e, f))
    buf = np.array(limbs(P) + limbs(Pp) + topc + [x for o in ops for v in o for x in (limbs(v) if v < R else limbs(v % R)[:-1] + [limbs(v % R)[-1] + (v >> (W * K)) * (1 << W)])], np.uint32)
    fin, fout = f"gpurun_out/r4k/in_{name}.bin", f"gpurun_out/r4k/out_{name}.bin"
    buf.tofile(fin)
    r = subprocess.run(["tools/dbg/wavedig_probe", fin, fout, str(n)], capture_output=True, text=True, timeout=120)
    print(name, r.returncode, r.stdout.strip(), r.stderr.strip()[-300:], flush=True)
    out = np.fromfile(fout, np.uint32).reshape(n, 2, K)
    rinv2 = pow(R * R, -1, P2)
    bad = []
    for i, (a, c, e, f) in enumerate(ops):
        ga, gc = val(out[i, 0]), val(out[i, 1])
        want = ((R * a + P * c) * (R * e + P * f) * rinv2) % P2
        m1 = (-a * e * pow(P, -1, R)) % R
        if (R * ga + P * gc) % P2 != want or ga != (a * e + m1 * P) // R:
            bad.append({"i": i, "a": hex(a), "c": hex(c), "e": hex(e), "f": hex(f), "ga": hex(ga), "gc": hex(gc),
                        "a_ok": ga == (a * e + m1 * P) // R})
    print(name, "bad", len(bad), "of", n, "by class", [sum(1 for b in bad if b["i"] % 4 == k) for k in range(4)], flush=True)
    json.dump(bad[:50], open(f"gpurun_out/r4k/bad_{name}.json", "w"))
