"""Debug: per-element decrypt results of the whole-wave digit path against
the oracle (batches of 7 and single elements), for the WaveDig bisection."""
import os, random, sys
sys.path.insert(0, os.getcwd())
from oracle import paillier_oracle as O
from tests.conftest import hx, load_fixture
from tests.test_gpu_parity import _dkey, _okey
from xfl_amd._native import ints_to_words, words_to_ints

g = load_fixture("paillier_2048_djn.json")
dk, ok = _dkey(g), _okey(g)
p, q, n = hx(g["key"]["p"]), hx(g["key"]["q"]), hx(g["key"]["n"])
n2 = n * n
rnd = random.Random(7)
cs = [1, n2 - 1, p * p - 1, p * p + 1, q * q - 2, q * q + 3, n + 1] + [rnd.randrange(1, n2) for _ in range(9)]
want = [O.decrypt_raw(ok, c) for c in cs]
out = words_to_ints(dk.decrypt_words(ints_to_words(cs, dk.n2w)))
print("batch", "".join("." if a == b else "X" for a, b in zip(out, want)), flush=True)
one = [words_to_ints(dk.decrypt_words(ints_to_words([c], dk.n2w)))[0] for c in cs]
print("single", "".join("." if a == b else "X" for a, b in zip(one, want)), flush=True)
# residues mod p^2 / q^2 separately: c with c = 1 mod q^2 (p-part only) and vice versa
crt = lambda a, b: (a * q * q * pow(q * q, -1, p * p) + b * p * p * pow(p * p, -1, q * q)) % n2
cp = [crt(rnd.randrange(1, p * p), 1) for _ in range(6)]
cq = [crt(1, rnd.randrange(1, q * q)) for _ in range(6)]
for name, xs in (("p-only", cp), ("q-only", cq)):
    w = [O.decrypt_raw(ok, c) for c in xs]
    o = words_to_ints(dk.decrypt_words(ints_to_words(xs, dk.n2w)))
    print(name, "".join("." if a == b else "X" for a, b in zip(o, w)), flush=True)
