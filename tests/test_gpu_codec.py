"""The device encoder (k_encode_f64) and decoder (k_decode) against the
reference's own outputs, on every golden input, through the C ABI.

Reference semantics pinned here:
  encode   encoder.py:29-54 (cal_exponent, round-half-even, wrap to n - |m|,
           the domain errors), paillier.py:279-282 (max_exponent clamp)
  decode   encoder.py:56-64 (signed range, OverflowError outside
           (max_pos, min_neg), mpfr RNE-53 product), paillier.py:396-403
           (astype(np.float32): the second rounding; mpz -> float overflow)
The expected m are the fixture's decrypted m (= the reference's encoded m),
the expected exponents and float64/float32 values its recorded outputs.
"""
import ctypes

import numpy as np
import pytest

from tests.conftest import FIXTURES, fl, hx, load_fixture

pytestmark = pytest.mark.gpu

FLOAT_CASES = ["priv_f32_p7", "pub_f32_p7", "priv_f64_none", "priv_edge_p7_noobf", "pub_f64_none_max-60"]
ST_OK, ST_OVERFLOW, ST_VALUE, ST_F32_OVERFLOW = 0, 1, 2, 3


def _dkey(g, private=True):
    from xfl_amd._native import DeviceKey
    k = g["key"]
    h = hx(k["h_pow_n"]) if k["djn_on"] else None
    if private:
        return DeviceKey(g["key_bits"], hx(k["n"]), hx(k["p"]), hx(k["q"]), h)
    return DeviceKey(g["key_bits"], hx(k["n"]), None, None, h)


def device_encode(dk, xs, precision, max_exponent):
    """xhe_encode_f64 on device buffers -> (m ints, exponents, statuses)."""
    import torch

    from xfl_amd import _native as nat
    n = len(xs)
    x = torch.tensor(np.asarray(xs, dtype=np.float64), device="cuda")
    m = torch.full((n, dk.nw), -1, dtype=torch.int32, device="cuda")
    e = torch.full((n,), 12345, dtype=torch.int32, device="cuda")
    st = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    prec = -1 if precision is None else int(precision)
    has_max = max_exponent is not None
    nat.check(nat.lib().xhe_encode_f64(dk.handle, x.data_ptr(), n, prec, int(has_max),
                                       int(max_exponent) if has_max else 0, m.data_ptr(), e.data_ptr(),
                                       st.data_ptr(), torch.cuda.current_stream().cuda_stream), "encode")
    torch.cuda.synchronize()
    return (nat.words_to_ints(m.cpu().numpy().view(np.uint32)), e.cpu().numpy().tolist(),
            st.cpu().numpy().tolist(), m)


def device_decode(dk, ms, exps):
    """xhe_decode on device buffers -> (float64 list, float32 array, statuses)."""
    import torch

    from xfl_amd import _native as nat
    n = len(ms)
    mw = torch.from_numpy(nat.ints_to_words(ms, dk.nw).view(np.int32).copy()).cuda()
    e = torch.tensor(exps, dtype=torch.int32, device="cuda")
    f64 = torch.full((n,), 7.0, dtype=torch.float64, device="cuda")
    f32 = torch.full((n,), 7.0, dtype=torch.float32, device="cuda")
    st = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    nat.check(nat.lib().xhe_decode(dk.handle, mw.data_ptr(), e.data_ptr(), n, f64.data_ptr(), f32.data_ptr(),
                                   st.data_ptr(), torch.cuda.current_stream().cuda_stream), "decode")
    torch.cuda.synchronize()
    return f64.cpu().numpy().tolist(), f32.cpu().numpy(), st.cpu().numpy().tolist()


def _f32hex(a):
    return [float(v).hex() for v in np.asarray(a, dtype=np.float32).astype(np.float64)]


@pytest.mark.parametrize("fx", FIXTURES)
@pytest.mark.parametrize("case", FLOAT_CASES)
def test_device_encode_golden(fx, case):
    """m and exponent per element equal the reference's: half-even ties at
    precision 7 (priv_edge_p7_noobf), frexp extremes 2^-960 / 1e-200-scale /
    2^52 at precision None, the max_exponent = -60 clamp, float32 inputs."""
    g = load_fixture(fx)
    enc = g["encrypt"][case]
    dec = g["decrypt"][case]
    dk = _dkey(g)
    xs = [fl(v) for v in enc["input"]]
    ms, es, st, _ = device_encode(dk, xs, enc["precision"], enc["max_exponent"])
    want_m = [hx(m) for m in dec["m"][len(dec["m"]) - len(xs):]]
    assert st == [ST_OK] * len(xs)
    assert es == enc["exp"]
    assert ms == want_m


@pytest.mark.parametrize("fx", FIXTURES)
def test_device_encode_errors(fx):
    """encode_errors_none: OverflowError (|x| below 2^-971, inf) and ValueError
    (NaN, positive exponent = negative shift count) exactly where the reference
    raised, as per-element statuses; and the drop-in raises those types."""
    from xfl_amd.paillier import Paillier, PaillierContext
    g = load_fixture(fx)
    dk = _dkey(g)
    cases = g["encrypt"]["encode_errors_none"]
    xs = [float(c["x"]) if c["x"] in ("inf", "-inf", "nan") else fl(c["x"]) for c in cases]
    _, _, st, _ = device_encode(dk, xs, None, None)
    want = [{"OverflowError": ST_OVERFLOW, "ValueError": ST_VALUE}[c["raises"]] for c in cases]
    assert st == want
    k = g["key"]
    ctx = PaillierContext().init(hx(k["p"]), hx(k["q"]), djn_h_pow_n=hx(k["h_pow_n"]) if k["djn_on"] else None)
    exc = {"OverflowError": OverflowError, "ValueError": ValueError}
    for x, c in zip(xs, cases):
        with pytest.raises(exc[c["raises"]]):
            Paillier.encrypt(ctx, np.array([1.0, x]), precision=None, obfuscation=False)
        with pytest.raises(exc[c["raises"]]):
            Paillier.encrypt(ctx, x, precision=None, obfuscation=False)


@pytest.mark.parametrize("fx", FIXTURES)
@pytest.mark.parametrize("case", FLOAT_CASES)
def test_device_encode_then_encrypt_bit_exact(fx, case):
    """Device encoder -> device encrypt with the reference's recorded draws
    (never touching the host encoder): ciphertexts equal the reference's."""
    import torch

    from xfl_amd import _native as nat
    g = load_fixture(fx)
    enc = g["encrypt"][case]
    dk = _dkey(g, private=enc["private"])
    xs = [fl(v) for v in enc["input"]]
    _, _, st, m_dev = device_encode(dk, xs, enc["precision"], enc["max_exponent"])
    assert st == [ST_OK] * len(xs)
    n = len(xs)
    ct = torch.empty((n, dk.n2w), dtype=torch.int32, device="cuda")
    r_dev = None
    if enc["obfuscation"]:
        r_dev = torch.from_numpy(nat.ints_to_words([hx(r) for r in enc["rand"]], dk.rand_words)
                                 .view(np.int32).copy()).cuda()
    nat.check(nat.lib().xhe_encrypt(dk.handle, m_dev.data_ptr(), r_dev.data_ptr() if r_dev is not None else None, n,
                                    ct.data_ptr(), torch.cuda.current_stream().cuda_stream), "encrypt")
    torch.cuda.synchronize()
    assert nat.words_to_ints(ct.cpu().numpy().view(np.uint32)) == [hx(r) for r in enc["raw"]]


@pytest.mark.parametrize("fx", FIXTURES)
def test_device_decode_crafted_and_overflow(fx):
    """decrypt.crafted: the double-rounding case (m = 2^54+2^30+1, e = -54 ->
    float64 1.0000001, float32 1.0), its negative, 2^e underflow, e >= 0
    integer decodes, mpz->float overflow (float32 'OverflowError');
    decrypt.overflow: OverflowError for max_pos < m < min_neg."""
    g = load_fixture(fx)
    dk = _dkey(g)
    crafted = g["decrypt"]["crafted"]
    f64, f32, st = device_decode(dk, [hx(c["m"]) for c in crafted], [c["exp"] for c in crafted])
    for i, c in enumerate(crafted):
        if c["float32"] == "OverflowError":
            assert st[i] == ST_F32_OVERFLOW, c
            continue
        assert st[i] == ST_OK, c
        origin = fl(c["origin"]) if ("p" in c["origin"] or "." in c["origin"]) else float(hx(c["origin"]))
        assert f64[i].hex() == origin.hex(), c
        assert _f32hex([f32[i]]) == [c["float32"]], c
    over = g["decrypt"]["overflow"]
    _, _, st = device_decode(dk, [hx(c["m"]) for c in over], [0] * len(over))
    assert st == [ST_OVERFLOW] * len(over)


@pytest.mark.parametrize("fx", FIXTURES)
@pytest.mark.parametrize("case", ["priv_f32_p7", "pub_f32_p7", "priv_f64_none", "priv_edge_p7_noobf",
                                  "pub_f64_none_max-60", "priv_packed_p0", "pub_i32_none"])
def test_decrypt_decode_host_golden(fx, case):
    """xhe_decrypt_decode_host (decrypt + decode + float32 in one call) on the
    reference's ciphertexts: float64 = the reference's out_origin value as a
    float, float32 = its Paillier.decrypt(dtype='float') output, bit for bit
    (packed ints decode to +-inf in float32, as numpy's cast gives)."""
    from xfl_amd import _native as nat
    g = load_fixture(fx)
    dk = _dkey(g)
    enc, dec = g["encrypt"][case], g["decrypt"][case]
    n = len(enc["raw"])
    cw = nat.ints_to_words([hx(r) for r in enc["raw"]], dk.n2w)
    ex = np.asarray(enc["exp"], dtype=np.int32)
    f64 = np.empty(n, np.float64)
    f32 = np.empty(n, np.float32)
    st = np.empty(n, np.int32)
    mo = np.empty((n, dk.nw), np.uint32)
    vp = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    nat.check(nat.lib().xhe_decrypt_decode_host(dk.handle, vp(cw), vp(ex), n, vp(f64), vp(f32), vp(st), vp(mo)))
    assert not st.any()
    assert nat.words_to_ints(mo) == [hx(m) for m in dec["m"][len(dec["m"]) - n:]]
    assert [float(v).hex() for v in f64] == dec["origin_f64"]
    assert _f32hex(f32) == dec["float32"]
