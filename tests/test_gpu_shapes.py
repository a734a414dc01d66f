"""The n^2 ciphertext operations run in two lane shapes chosen by batch size
(one 16-lane DPP row per residue up to 4,096 elements, 4 lanes beyond): add
with exponent alignment, scalar powers (both signs), batch inversion,
segmented products and multi-exponentiation give the same values in both
shapes and match Python's pow arithmetic (the reference's gmpy2 semantics,
utils.py:46-76) on sampled elements."""
import random

import numpy as np
import pytest

from tests.conftest import FIXTURES, hx, load_fixture

pytestmark = pytest.mark.gpu

BIG, SMALL = 4200, 60  # 4-lane shape / 16-lane shape


@pytest.fixture(scope="module", params=FIXTURES)
def ctx(request):
    from xfl_amd.paillier import PaillierContext
    k = load_fixture(request.param)["key"]
    return PaillierContext().init(hx(k["p"]), hx(k["q"])).to_public()


def _rand_cts(ctx, n, seed):
    rng = random.Random(seed)
    return [rng.randrange(1, ctx.n_square) for _ in range(n)]


def test_add_aligned_both_shapes(ctx):
    from xfl_amd.paillier import ops
    n2 = ctx.n_square
    ra, rb = _rand_cts(ctx, BIG, 1), _rand_cts(ctx, BIG, 2)
    rng = np.random.default_rng(3)
    ea = rng.integers(-30, -20, BIG).astype(np.int32)
    eb = rng.integers(-30, -20, BIG).astype(np.int32)
    big, ebig = ops.add(ctx, ra, ea, rb, eb)
    small, esmall = ops.add(ctx, ra[:SMALL], ea[:SMALL], rb[:SMALL], eb[:SMALL])
    assert small == big[:SMALL] and list(esmall) == list(ebig[:SMALL])
    for i in (0, 7, SMALL - 1, BIG - 1):
        e = min(ea[i], eb[i])
        want = pow(ra[i], 1 << int(ea[i] - e), n2) * pow(rb[i], 1 << int(eb[i] - e), n2) % n2
        assert big[i] == want and ebig[i] == e


@pytest.mark.parametrize("invert_first", [False, True])
def test_powmod_both_shapes(ctx, invert_first):
    from xfl_amd.paillier import ops
    n2 = ctx.n_square
    rs = _rand_cts(ctx, BIG, 4)
    rng = random.Random(5)
    ks = [rng.getrandbits(rng.choice([1, 20, 53, 75])) for _ in range(BIG)]
    big = ops.powmod(ctx, rs, ks, invert_first=invert_first)
    small = ops.powmod(ctx, rs[:SMALL], ks[:SMALL], invert_first=invert_first)
    assert small == big[:SMALL]
    for i in (0, 3, SMALL - 1, BIG - 1):
        base = pow(rs[i], -1, n2) if invert_first else rs[i]
        assert big[i] == pow(base, ks[i], n2)


def test_segment_sums_both_shapes(ctx):
    from xfl_amd.paillier import ops
    n2 = ctx.n_square
    for n in (BIG, SMALL):
        rs = _rand_cts(ctx, n, 6)
        exps = np.zeros(n, dtype=np.int64)
        exps[::3] = -1
        cuts = sorted(random.Random(7).sample(range(1, n), 9))
        seg = np.array([0] + cuts + [n], dtype=np.int64)
        got, emin = ops.segment_sums(ctx, rs, exps, seg)
        for s in (0, 4, 9):
            lo, hi = int(seg[s]), int(seg[s + 1])
            want = 1
            for i in range(lo, hi):
                want = want * pow(rs[i], 1 << int(exps[i] - emin[s]), n2) % n2
            assert got[s] == want


@pytest.mark.parametrize("nbases,ncols", [(24, 5), (BIG + 100, 2)])
def test_multiexp_both_shapes(ctx, nbases, ncols):
    from xfl_amd.paillier import ops
    n2 = ctx.n_square
    bases = _rand_cts(ctx, nbases, 8)
    rng = random.Random(9)
    nterms = min(nbases, 40)
    idx = [[rng.randrange(nbases) for _ in range(nterms)] for _ in range(ncols)]
    ks = [[rng.getrandbits(60) for _ in range(nterms)] for _ in range(ncols)]
    got = ops.multiexp(ctx, bases, idx, ks)
    for j in range(ncols):
        want = 1
        for t in range(nterms):
            want = want * pow(bases[idx[j][t]], ks[j][t], n2) % n2
        assert got[j] == want


def test_djn_encrypt_both_shapes():
    """DJN private encryption: the 16-lane small-batch kernel (k_djn_pow_x, on
    the one-lane tables with the (R'/R)^nwin start factor) and the one-lane
    kernel give identical ciphertexts, equal to the closed form - with uniform
    windows and with split layouts (XHE_WIN_SPLIT: the first rand_bits mod w
    windows w+1 bits wide, their tables built as a second segment)."""
    from oracle import paillier_oracle as O
    from xfl_amd._native import XHE_WIN_SPLIT, DeviceKey, ints_to_words, win_layout, words_to_ints
    for fx in FIXTURES:
        g = load_fixture(fx)
        k = g["key"]
        if not k["djn_on"]:
            continue
        n, p, q, h = hx(k["n"]), hx(k["p"]), hx(k["q"]), hx(k["h_pow_n"])
        for win in (16, 7, 7 | XHE_WIN_SPLIT, 10 | XHE_WIN_SPLIT):
            if win & XHE_WIN_SPLIT:
                assert win_layout(g["key_bits"] // 2, win)[1] > 0  # really split
            dk = DeviceKey(g["key_bits"], n, p, q, h, win_bits=win)
            rng = random.Random(win)
            nbig = 24000  # above the 16-lane encryption limit (20,480)
            ms = [rng.randrange(n) for _ in range(nbig)]
            rs = [rng.randrange(1, 1 << dk.rand_bits) for _ in range(nbig)]
            mw, rw = ints_to_words(ms, dk.nw), ints_to_words(rs, dk.rand_words)
            big = words_to_ints(dk.encrypt_words(mw, rw))
            small = words_to_ints(dk.encrypt_words(mw[:SMALL], rw[:SMALL]))
            assert small == big[:SMALL]
            # 2048 bits (Montgomery-digit kernel): 16 lanes per element up to
            # 2 k elements, 4 up to 16 k, 1 beyond - three splits of the windows
            mid = words_to_ints(dk.encrypt_words(mw[:3000], rw[:3000]))
            assert mid == big[:3000]
            ok = O.derive_private(p, q, h)
            for i in (0, SMALL - 1, 2999, nbig - 1):
                assert big[i] == O.encrypt_m(ok, ms[i], rs[i])


@pytest.mark.parametrize("fx", ["paillier_2048_djn.json", "paillier_3072_djn.json", "paillier_4096_djn.json"])
def test_private_nodjn_encrypt_closed_form(fx):
    """Private-key non-DJN encryption (r^ep mod p^2, r^eq mod q^2, CRT;
    paillier.py:214-230) equals the closed form (1 + n m) r^n mod n^2 —
    at 3072 bits it runs in the 4-lane shape, not the 2-lane batch shape."""
    from xfl_amd import _native as nat
    k = load_fixture(fx)["key"]
    p, q = hx(k["p"]), hx(k["q"])
    n = p * q
    n2 = n * n
    dk = nat.DeviceKey(int(fx.split("_")[1]), n, p, q, None, device=0)
    rng = random.Random(11)
    count = 2000
    ms = [rng.randrange(n) for _ in range(count)]
    rs = [rng.randrange(1, n) for _ in range(count)]
    ct = nat.words_to_ints(dk.encrypt_words(nat.ints_to_words(ms, dk.nw), nat.ints_to_words(rs, dk.rand_words)))
    for i in list(range(4)) + [count - 1]:
        assert ct[i] == (1 + n * ms[i]) * pow(rs[i], n, n2) % n2, i
    assert nat.words_to_ints(dk.decrypt_words(nat.ints_to_words(ct, dk.n2w))) == ms


@pytest.mark.parametrize("fx", ["paillier_2048_djn.json", "paillier_3072_djn.json", "paillier_4096_djn.json"])
def test_public_nodjn_encrypt_closed_form(fx):
    """Public-key encryption without h^n (the remote party's mode,
    context.py:152-168; paillier.py:228-230): (1 + n m) r^n mod n^2 with the
    exponent n walked by the wave-uniform sliding window."""
    from xfl_amd import _native as nat
    k = load_fixture(fx)["key"]
    n = hx(k["n"])
    n2 = n * n
    dk = nat.DeviceKey(int(fx.split("_")[1]), n, None, None, None, device=0)
    rng = random.Random(12)
    count = 1500
    ms = [rng.randrange(n) for _ in range(count)]
    rs = [rng.randrange(1, n) for _ in range(count)]
    ct = nat.words_to_ints(dk.encrypt_words(nat.ints_to_words(ms, dk.nw), nat.ints_to_words(rs, dk.rand_words)))
    for i in list(range(4)) + [count // 2, count - 1]:
        assert ct[i] == (1 + n * ms[i]) * pow(rs[i], n, n2) % n2, i


@pytest.mark.parametrize("fx", ["paillier_3072_djn.json", "paillier_4096_djn.json"])
def test_decrypt_digits_batch(fx):
    """3072/4096-bit decrypt of batches above the 16-lane limit (5,120) runs in
    Montgomery digits of P (k_p2_reduce_words, k_dec_pmdx_in/pow/out): the
    round trip of 6,000 device encryptions is bit-exact, and arbitrary
    residues mod n^2 (not ciphertexts) decrypt as the oracle's
    L(c^(p-1) mod p^2) hp mod p with CRT (paillier.py:341-368)."""
    from oracle import paillier_oracle as O
    from xfl_amd import _native as nat
    g = load_fixture(fx)
    k = g["key"]
    p, q, h = hx(k["p"]), hx(k["q"]), hx(k["h_pow_n"])
    n = p * q
    dk = nat.DeviceKey(g["key_bits"], n, p, q, h, device=0, win_bits=10)
    rng = random.Random(13)
    count = 6000
    ms = [rng.randrange(n) for _ in range(count)]
    rs = [rng.randrange(1, 1 << dk.rand_bits) for _ in range(count)]
    ct = dk.encrypt_words(nat.ints_to_words(ms, dk.nw), nat.ints_to_words(rs, dk.rand_words))
    assert nat.words_to_ints(dk.decrypt_words(ct)) == ms
    ok = O.derive_private(p, q, h)
    cs = [rng.randrange(1, n * n) for _ in range(count)]
    cs[:3] = [1, n * n - 1, n + 1]
    got = nat.words_to_ints(dk.decrypt_words(nat.ints_to_words(cs, dk.n2w)))
    for i in (0, 1, 2, 3, 2047, count - 1):
        assert got[i] == O.decrypt_raw(ok, cs[i]), i


_PIN_SCRIPT = r"""
import sys
sys.path.insert(0, {root!r})
import torch
torch.cuda.init()
from tests.conftest import hx, load_fixture
from xfl_amd import _native as nat
g = load_fixture({fx!r})
k = g["key"]
p, q, h = hx(k["p"]), hx(k["q"]), hx(k["h_pow_n"])
dk = nat.DeviceKey(g["key_bits"], p * q, p, q, h, device=0, win_bits=8)
cts, want = [], []
for case, enc in g["encrypt"].items():
    if not isinstance(enc, dict) or case not in g["decrypt"]:
        continue
    dec = g["decrypt"][case]
    cts += [hx(r) for r in enc["raw"]]
    want += [hx(m) for m in dec["m"][len(dec["m"]) - len(enc["raw"]):]]
got = nat.words_to_ints(dk.decrypt_words(nat.ints_to_words(cts, dk.n2w)))
assert got == want, "golden decrypt differs"
print("ok", len(got))
"""


@pytest.mark.parametrize("fx", ["paillier_3072_djn.json", "paillier_4096_djn.json"])
def test_decrypt_digits_golden_pinned(fx):
    """Every golden ciphertext of the 3072/4096-bit fixtures decrypts to the
    reference's m through the digit kernels ($XHE_DEC_TPI=1 pins them for
    small batches; the pin is read once per process, hence the child)."""
    import os
    import subprocess
    import sys

    from tests.conftest import ROOT
    env_ = dict(os.environ, XHE_DEC_TPI="1")
    r = subprocess.run([sys.executable, "-c", _PIN_SCRIPT.format(root=ROOT, fx=fx)], env=env_, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout[-2000:] + r.stderr[-3000:]
