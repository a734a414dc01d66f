"""CPU: the plaintext-side restatement used to check the LR HE round
(tools/lr_he_demo.expected_noised_gradient) equals the oracle's ciphertext
path (encrypt -> per-element mul/add fold -> scalar add -> decrypt -> decode,
paillier.py:106-187, 341-398) on the golden 2048-bit DJN key."""
import random

import numpy as np

from oracle import paillier_oracle as O
from tests.conftest import FIXTURES, hx, load_fixture


def test_restatement_matches_ciphertext_path():
    from tools.lr_he_demo import expected_noised_gradient, load_wdbc
    k = load_fixture(FIXTURES[0])["key"]
    ok = O.derive_private(hx(k["p"]), hx(k["q"]), hx(k["h_pow_n"]))
    xtr, ytr, _, _ = load_wdbc()
    B, D = 6, 3
    x = xtr[:B, 15:15 + D]
    resid = (ytr[:B] - np.float32(0.37)).astype(np.float32)
    noise = np.array([0.125, -3.5e-4, 201.0], dtype=np.float32)
    rng = random.Random(1)
    cts = []
    for r in resid:
        m, e = O.encode_element(ok, float(r), 7)
        cts.append((O.encrypt_m(ok, m, rng.randrange(1, ok["djn_exp_bound"])), e))
    got = []
    for j in range(D):
        acc = None
        for (c, e), xv in zip(cts, x[:, j]):
            t = O.mul_ct(ok, c, e, xv.item())
            acc = t if acc is None else O.add_ct(ok, acc[0], acc[1], t[0], t[1])
        c, e = O.add_scalar(ok, acc[0], acc[1], float(noise[j]))
        got.append(O.decode_float32(ok, O.decrypt_raw(ok, c), e))
    want = expected_noised_gradient(ok, resid, x, noise)
    assert np.array_equal(np.array(got, dtype=np.float32).view(np.uint32), want.view(np.uint32))
