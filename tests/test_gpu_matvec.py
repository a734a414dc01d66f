"""Encrypted mat-vec (np.matmul(enc[B], X[B, D]), logistic_regression/trainer.py:166)
through the multi-exponentiation kernels (xhe_multiexp), bit-exact against the
oracle's left fold of the reference's own per-element operations
(paillier.py:106-187: mul by a float scalar, then add with exponent alignment).

The key is the golden 2048-bit DJN fixture key; ciphertexts are random
residues mod n^2 coprime to n (what a real encryption is), so the result does
not depend on obfuscation draws. Sizes are ragged and X mixes magnitudes,
signs and exact zeros, so every term class of the reference is hit:
positive/negative scalars (inverse branch), exponent alignment across rows,
and 0 * c (exponent -53, raw 1).
"""
import random

import numpy as np
import pytest

from oracle import paillier_oracle as O
from tests.conftest import FIXTURES, hx, load_fixture

pytestmark = pytest.mark.gpu


def _keys(fx):
    from xfl_amd.paillier import PaillierContext
    g = load_fixture(fx)
    k = g["key"]
    h = hx(k["h_pow_n"]) if k["djn_on"] else None
    priv = PaillierContext().init(hx(k["p"]), hx(k["q"]), djn_h_pow_n=h)
    return priv, O.derive_private(hx(k["p"]), hx(k["q"]), h)


def _oracle_matmul(ok, raws, exps, X):
    out = []
    for j in range(X.shape[1]):
        acc = None
        for i in range(X.shape[0]):
            t = O.mul_ct(ok, raws[i], exps[i], X[i, j].item())
            acc = t if acc is None else O.add_ct(ok, acc[0], acc[1], t[0], t[1])
        out.append(acc)
    return out


@pytest.mark.parametrize("fx", [FIXTURES[0], FIXTURES[2]])
@pytest.mark.parametrize("B, D", [(1, 1), (37, 3), (130, 5)])
def test_matmul_bit_exact_vs_oracle(fx, B, D):
    from xfl_amd.paillier import PaillierArray, PaillierCiphertext
    priv, ok = _keys(fx)
    pub = priv.to_public()
    rng = random.Random(B * 1000 + D)
    n2 = ok["n_square"]
    raws = []
    while len(raws) < B:
        c = rng.randrange(2, n2)
        if c % ok["p"] and c % ok["q"]:
            raws.append(c)
    exps = [rng.choice([-24, -53, -60, 0]) for _ in range(B)]
    nrng = np.random.default_rng(B + D)
    X = (nrng.standard_normal((B, D)) * np.exp2(nrng.integers(-12, 6, (B, D)))).astype(np.float32)
    X[nrng.random((B, D)) < 0.1] = 0.0
    X[0, 0] = -1.0
    A = PaillierArray(np.array([PaillierCiphertext(pub, r, e) for r, e in zip(raws, exps)], dtype=object))
    got = np.matmul(A, X)
    want = _oracle_matmul(ok, raws, exps, X)
    assert [(c.raw_ciphertext, c.exponent) for c in got] == want


def test_multiexp_abi_direct():
    """xhe_multiexp_host with repeated bases, a one-term column and k = 0."""
    from xfl_amd.paillier import ops
    priv, ok = _keys(FIXTURES[0])
    n2 = ok["n_square"]
    rng = random.Random(5)
    bases = [rng.randrange(2, n2) for _ in range(6)]
    idx = [[0, 1, 2, 3, 4, 5, 0], [5, 5, 5, 5, 5, 5, 5], [3, 3, 1, 1, 0, 0, 2]]
    ks = [[rng.getrandbits(70) for _ in range(7)], [0] * 7, [1, 2, 3, 0, 1 << 69, 7, 1]]
    got = ops.multiexp(priv, bases, idx, ks)
    for j in range(3):
        want = 1
        for t in range(7):
            want = want * pow(bases[idx[j][t]], ks[j][t], n2) % n2
        assert got[j] == want
