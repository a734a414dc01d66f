"""The drop-in package (xfl_amd.paillier) against the reference's outputs.

Homomorphic operations are checked bit-exactly against the golden vectors
(tests/golden, produced by XFL's own code); randomized encryption is checked
through decryption, with the same tolerances as the reference's tests
(test/common/crypto/paillier/test_paillier.py).
"""
import random

import numpy as np
import pytest

from tests.conftest import FIXTURES, fl, hx, load_fixture

pytestmark = pytest.mark.gpu


from tests import dropin_cases as C


@pytest.mark.parametrize("vectorized", [False, True, "resident"])
@pytest.mark.parametrize("fx", FIXTURES)
def test_ops_bit_exact(fx, vectorized):
    C.ops_bit_exact(fx, vectorized)


def test_histogram_groupby_bit_exact():
    C.histogram_groupby(FIXTURES[0])


@pytest.mark.parametrize("vectorized", [False, True, "resident"])
@pytest.mark.parametrize("fx", ["paillier_2048_djn.json", "paillier_2048_nodjn.json"])
def test_gap_alignment_negative_branch(fx, vectorized):
    """device alignment across gaps >= the negative-branch threshold:
    xhe_mulmod's fix-up (vectorized adds) and the tree-aware segmented
    product (np.sum, Python sum, deferred object adds)"""
    C.gap_alignment(fx, vectorized)


def test_mulmod_gap_c_abi():
    """xhe_mulmod itself (device buffers) reproduces _raw_mul's negative
    branch for every gap case of the fixture, mixed with small gaps in one call"""
    import torch

    from xfl_amd import _native as nat
    g = load_fixture("paillier_2048_djn.json")
    priv, pub = C.ctxs(g)
    ops = g["ops"]
    dk = pub.device_key()
    ops_raw = [hx(r) for r in ops["gap_operands"]["raw"]]
    ops_exp = ops["gap_operands"]["exp"]
    pairs = ops["gap"]["pairs"]
    a = torch.from_numpy(nat.ints_to_words([ops_raw[i] for i, _ in pairs], dk.n2w).view(np.int32).copy()).cuda()
    b = torch.from_numpy(nat.ints_to_words([ops_raw[j] for _, j in pairs], dk.n2w).view(np.int32).copy()).cuda()
    ea = torch.tensor([ops_exp[i] for i, _ in pairs], dtype=torch.int32).cuda()
    eb = torch.tensor([ops_exp[j] for _, j in pairs], dtype=torch.int32).cuda()
    out = torch.empty_like(a)
    eo = torch.empty_like(ea)
    dmax = int((ea - eb).abs().max().item())
    s = torch.cuda.current_stream().cuda_stream
    nat.check(nat.lib().xhe_mulmod(dk.handle, a.data_ptr(), ea.data_ptr(), b.data_ptr(), eb.data_ptr(), len(pairs),
                                   dmax, out.data_ptr(), eo.data_ptr(), s), "mulmod")
    torch.cuda.synchronize()
    assert nat.words_to_ints(out.cpu().numpy().view(np.uint32)) == [hx(r) for r in ops["gap_add_pub"]["raw"]]
    assert eo.tolist() == ops["gap_add_pub"]["exp"]
    # one exponent array NULL (= all 0, include/xhe.h): the same gaps relative
    # to it take the same negative branch (the fix runs whenever dmax >= dneg)
    want = [hx(r) for r in ops["gap_add_pub"]["raw"]]
    for null_a in (True, False):
        rel = (eb - ea) if null_a else (ea - eb)
        nat.check(nat.lib().xhe_mulmod(dk.handle, a.data_ptr(), None if null_a else rel.data_ptr(), b.data_ptr(),
                                       rel.data_ptr() if null_a else None, len(pairs), dmax, out.data_ptr(),
                                       eo.data_ptr(), s), "mulmod")
        torch.cuda.synchronize()
        assert nat.words_to_ints(out.cpu().numpy().view(np.uint32)) == want, null_a
        shift = ea if null_a else eb
        assert eo.tolist() == [e - int(d) for e, d in zip(ops["gap_add_pub"]["exp"], shift.tolist())]


@pytest.mark.parametrize("fx", FIXTURES)
def test_decrypt_matches_reference(fx):
    C.decrypt_matches_reference(fx)


@pytest.mark.parametrize("fx", FIXTURES)
def test_wire_roundtrip_with_reference_pickles(fx):
    C.wire_roundtrip(fx)


@pytest.mark.parametrize("resident", [False, True])
@pytest.mark.parametrize("fx", FIXTURES[:2])
def test_array_protocol(fx, resident):
    C.array_protocol(fx, resident)


@pytest.mark.parametrize("fx", FIXTURES)
def test_encrypt_decrypt_shapes(fx):
    C.encrypt_decrypt_shapes(fx)


def _ctxs(g):
    return C.ctxs(g)


# ---- ports of the reference's tolerance tests (test_paillier.py:24-296)
data = [(True, None, True, -1), (True, 7, True, -1), (True, 7, False, 1),
        (False, None, True, -1), (False, 7, True, -1), (False, 7, False, 1)]


@pytest.fixture(scope="module")
def ctx():
    from xfl_amd.paillier import PaillierContext
    return PaillierContext.generate(2048)


@pytest.mark.parametrize("djn_on, precision, is_batch, num_cores", data)
def test_unary(ctx, djn_on, precision, is_batch, num_cores):
    from xfl_amd.paillier import Paillier
    p1 = np.random.random((50,)).astype(np.float32) * 100 - 50 if is_batch else random.random() * 100 - 50
    c1 = Paillier.encrypt(ctx, p1, precision=precision, max_exponent=None, obfuscation=True, num_cores=num_cores)
    pub = ctx.to_public()
    c11 = Paillier.encrypt(pub, p1, precision=precision, max_exponent=None, obfuscation=True, num_cores=num_cores)
    a = Paillier.decrypt(ctx, c1, num_cores=num_cores)
    assert np.all(np.abs(a - p1) < 1e-4)
    b = Paillier.decrypt(ctx, c11, num_cores=num_cores)
    assert np.all(np.abs(b - p1) < 1e-4)
    with pytest.raises(TypeError):
        Paillier.decrypt(pub, c1, num_cores=num_cores)


@pytest.mark.parametrize("djn_on, precision, is_batch, num_cores", data)
def test_binary(ctx, djn_on, precision, is_batch, num_cores):
    from xfl_amd.paillier import Paillier
    if is_batch:
        p1 = np.random.random((50,)).astype(np.float32) * 100 - 50
        p2 = np.random.random((50,)).astype(np.float32) * 100 - 20
    else:
        p1 = random.random() * 100 - 50
        p2 = random.random() * 100 - 20
    c1 = Paillier.encrypt(ctx, p1, precision=precision, obfuscation=True, num_cores=num_cores)
    c2 = Paillier.encrypt(ctx, p2, precision=precision, obfuscation=True, num_cores=num_cores)
    eps = 1e-4
    if is_batch:
        assert abs(Paillier.decrypt(ctx, sum(c1)) - np.sum(p1.astype(np.float64))) < 1e-2
    assert np.all(np.abs(Paillier.decrypt(ctx, c1 + c2) - (p1 + p2)) < eps)
    assert np.all(np.abs(Paillier.decrypt(ctx, c1 - c2) - (p1 - p2)) < eps)
    assert np.all(np.abs(Paillier.decrypt(ctx, c1 + p2) - (p1 + p2)) < eps)
    assert np.all(np.abs(Paillier.decrypt(ctx, c1 - p2) - (p1 - p2)) < eps)
    assert np.all(np.abs(Paillier.decrypt(ctx, p2 - c1) - (p2 - p1)) < eps)
    assert np.all(np.abs(Paillier.decrypt(ctx, c1 * p2) - (p1 * p2)) < 1e-2)
    assert np.all(np.abs(Paillier.decrypt(ctx, c1 / p2) - (p1 / p2)) < eps)


def test_rest_errors_and_djn():
    from xfl_amd.paillier import Paillier, PaillierCiphertext
    context = Paillier.context(2048)
    p1 = random.random() * 100 - 50
    c1 = Paillier.encrypt(context, p1, precision=7, max_exponent=None, obfuscation=True)
    for comp in (True, False):
        s = c1.serialize(comp)
        c2 = PaillierCiphertext.deserialize_from(context, s, comp)
        assert c1.raw_ciphertext == c2.raw_ciphertext and c1.exponent == c2.exponent
    with pytest.raises(TypeError):
        c1 + "342"
    other = Paillier.context(2048)
    c3 = Paillier.encrypt(other, p1, precision=7)
    with pytest.raises(ValueError):
        c1 + c3
    with pytest.raises(TypeError):
        c1 * c1
    pub = context.to_public()
    c1 = Paillier.obfuscate(Paillier.encrypt(pub, p1, precision=7))
    assert abs(Paillier.decrypt(context, c1) - p1) < 1e-5
    djn = Paillier.context(2048, djn_on=True)
    assert abs(Paillier.decrypt(djn, Paillier.encrypt(djn, p1, precision=7)) - p1) < 1e-5
    dpub = djn.to_public()
    assert abs(Paillier.decrypt(djn, Paillier.encrypt(dpub, p1, precision=7)) - p1) < 1e-5
    c = Paillier.encrypt(dpub, p1, precision=7, max_exponent=20, obfuscation=False)
    assert abs(Paillier.decrypt(djn, c, num_cores=1) - p1) < 1e-5
    with pytest.raises(TypeError):
        Paillier.encrypt(dpub, "123", precision=7)
    c3 = Paillier.obfuscate(Paillier.encrypt(dpub, 3, precision=7))
    assert Paillier.decrypt(djn, c3, dtype="int") == 3
    p4 = np.array([2, 3], dtype=np.int32)
    c4 = Paillier.obfuscate(Paillier.encrypt(dpub, p4, precision=7))
    assert np.all(Paillier.decrypt(djn, c4, dtype="int") == p4)
    assert 123 == Paillier._decrypt_single(123, djn)
    with pytest.raises(TypeError):
        Paillier.decrypt(djn, 123)
    with pytest.raises(TypeError):
        Paillier.obfuscate(123)


def test_deferred_sums_groupby_and_chains():
    """pandas groupby sum / np.sum / sum() over object columns build deferred
    sums (one segmented-product call when read); results equal the oracle's
    aligned product, including mixed exponents and shared operands."""
    import time

    import pandas as pd

    from oracle import paillier_oracle as O
    from xfl_amd.paillier import PaillierCiphertext
    g = load_fixture(FIXTURES[0])
    priv, pub = _ctxs(g)
    k = g["key"]
    ok = O.derive_private(hx(k["p"]), hx(k["q"]), hx(k["h_pow_n"]))
    rng = random.Random(9)
    n2 = ok["n_square"]
    N, NB = 3000, 32
    raws = [rng.randrange(2, n2) for _ in range(N)]
    exps = [rng.choice([0, -3, -7]) for _ in range(N)]
    bins = [rng.randrange(NB) for _ in range(N)]
    cts = [PaillierCiphertext(pub, r, e) for r, e in zip(raws, exps)]
    t = time.time()
    df = pd.DataFrame({"bin": bins, "c": np.array(cts, dtype=object)})
    agg = df.groupby(["bin"])["c"].agg(["count", "sum"])
    got = [(c.raw_ciphertext, c.exponent) for c in agg["sum"]]
    elapsed = time.time() - t
    for b in range(NB):
        idx = [i for i in range(N) if bins[i] == b]
        assert got[b] == O.sum_ct(ok, [raws[i] for i in idx], [exps[i] for i in idx])
    assert elapsed < 30, f"groupby over {N} ciphertexts took {elapsed:.1f}s"
    # a chain reusing one operand, then an eager op on the deferred result
    s = cts[0] + cts[1]
    s2 = s + cts[0] + s
    want = O.sum_ct(ok, [raws[0], raws[1], raws[0], raws[0], raws[1]], [exps[0], exps[1], exps[0], exps[0], exps[1]])
    assert (s2.raw_ciphertext, s2.exponent) == want
    m = s2 * 3
    assert m.raw_ciphertext == O.mul_ct(ok, want[0], want[1], 3)[0]


@pytest.mark.parametrize("fx", ["paillier_3072_djn.json", "paillier_4096_djn.json", "paillier_8192_djn.json"])
def test_larger_keys_tolerance_ops(fx):
    """The reference's tolerance checks (test_paillier.py:24-296) on the
    3072/4096/8192-bit fixture keys (the operators offer key_bit_size 4096/8192,
    config_descriptor/vertical_logistic_regression/label_trainer.py:118):
    private and public encryption, +, -, scalar *, / and the batch sum, in
    batches large enough to take the one-lane-per-residue kernels."""
    from xfl_amd.paillier import Paillier
    priv, pub = _ctxs(load_fixture(fx))
    rng = np.random.default_rng(5)
    p1 = (rng.random(30000) * 100 - 50).astype(np.float32)
    p2 = (rng.random(30000) * 100 - 20).astype(np.float32)
    c1 = Paillier.encrypt(priv, p1, precision=7)
    c2 = Paillier.encrypt(pub, p2, precision=7)
    assert np.all(np.abs(Paillier.decrypt(priv, c1) - p1) < 1e-4)
    assert np.all(np.abs(Paillier.decrypt(priv, c2) - p2) < 1e-4)
    s1, s2, c1s, c2s = p1[:64], p2[:64], c1[:64], c2[:64]
    assert np.all(np.abs(Paillier.decrypt(priv, c1s + c2s) - (s1 + s2)) < 1e-4)
    assert np.all(np.abs(Paillier.decrypt(priv, c1s - c2s) - (s1 - s2)) < 1e-4)
    assert np.all(np.abs(Paillier.decrypt(priv, c1s * s2) - (s1 * s2)) < 1e-2)
    assert np.all(np.abs(Paillier.decrypt(priv, c1s / s2) - (s1 / s2)) < 1e-4)
    assert abs(Paillier.decrypt(priv, sum(c1s)) - np.sum(s1.astype(np.float64))) < 1e-2


@pytest.mark.parametrize("ctx_kind", ["pub", "priv"])
def test_add_plain_aligned_bit_exact(ctx_kind):
    """ciphertext + plaintext array on the device path, bit-exact against the
    reference's encrypt-then-align (paillier.py:95-123, oracle.add_scalar):
    plaintexts whose exponent is above the ciphertext's (the scalar encoded at
    the ciphertext's exponent, m 2^d, gaps from 1 to ~1,000 bits), below it
    (the ciphertext is raised), equal, zero, negative, ints and scalars; a
    ciphertext at exponent -2076 takes the encrypt-then-align path (m 2^d past
    n); |x| >= 2^53 raises as the reference's encoder does."""
    from oracle import paillier_oracle as O
    from xfl_amd.paillier import PaillierArray
    g = load_fixture("paillier_2048_djn.json")
    priv, pub = C.ctxs(g)
    ctx = pub if ctx_kind == "pub" else priv
    ok = O.derive_private(priv.p, priv.q, priv.h_pow_n)
    rng = np.random.default_rng(3)
    p = np.array([123.25, -7.5, 0.0, 1e-30, -3e-25, 2.0 ** 52 + 1, -4.5e15, 335.0, -0.001, 2.0 ** -600, 1.0, -1.0])
    p32 = p.astype(np.float32)
    base = C.cts(ctx, g["encrypt"]["priv_f32_p7"])[:1]  # exponent -24
    A0 = PaillierArray(np.array([base[0]] * 12, dtype=object))
    A0.to_device()
    deep = A0 * (2.0 ** -900)  # exponent -976: gaps of ~930 bits
    far = PaillierArray(np.array(C.cts(ctx, g["ops"]["gap_operands"])[:1].tolist() * 12, dtype=object))
    far.to_device()  # exponent -2076
    for A in (A0, deep, far):
        raws, exps = C.raw(A)
        for P in (p, p32, rng.integers(-1000, 1000, 12).astype(np.int64)):
            got = A + P
            want = [O.add_scalar(ok, r, e, v.item()) for r, e, v in zip(raws, exps, P)]
            assert C.raw(got) == ([w[0] for w in want], [w[1] for w in want])
        for sc in (3.75, -2.5e-9, 7):
            got = A + sc
            want = [O.add_scalar(ok, r, e, sc) for r, e in zip(raws, exps)]
            assert C.raw(got) == ([w[0] for w in want], [w[1] for w in want])
        with pytest.raises(ValueError):
            A + np.full(12, 1e300)
