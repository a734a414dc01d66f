"""Host-side logic of the drop-in (no GPU): encoder/decoder semantics, context
derivation, wire compatibility, key generation helpers."""
import numpy as np
import pytest

from tests.conftest import FIXTURES, fl, hx, load_fixture


def test_context_derivation_matches_reference(golden):
    from xfl_amd.paillier import PaillierContext
    k = golden["key"]
    h = hx(k["h_pow_n"]) if k["djn_on"] else None
    ctx = PaillierContext().init(hx(k["p"]), hx(k["q"]), djn_h_pow_n=h)
    for name in ("q_inverse_p", "p_square", "q_square", "q2_inverse_p2", "hp", "hq", "phi_p2", "phi_q2", "ep", "eq",
                 "n_square", "max_value_for_positive", "min_value_for_negative"):
        assert getattr(ctx, name) == hx(k[name]), name
    if k["djn_on"]:
        assert ctx.djn_exp_bound == hx(k["djn_exp_bound"])
        assert ctx.h_pow_n_modp2 == hx(k["h_pow_n_modp2"])
    pub = ctx.to_public()
    assert not pub.is_private() and pub.n == ctx.n and pub.p is None
    assert PaillierContext.deserialize_from(ctx.serialize()) == ctx
    assert PaillierContext.deserialize_from(ctx.serialize(save_private_key=False)) != ctx
    with pytest.raises(ValueError):
        PaillierContext().init()
    PaillierContext().init(3, 5, 10)


def test_decode_single_matches_reference(golden):
    from xfl_amd.paillier import PaillierContext, PaillierEncoder
    k = golden["key"]
    ctx = PaillierContext().init(hx(k["p"]), hx(k["q"]))
    for rec in golden["decrypt"]["crafted"]:
        v = PaillierEncoder.decode_single(ctx, hx(rec["m"]), rec["exp"])
        if rec["exp"] < 0:
            assert v.hex() == rec["origin"]
        else:
            assert v == hx(rec["origin"])
    for rec in golden["decrypt"]["overflow"]:
        with pytest.raises(OverflowError):
            PaillierEncoder.decode_single(ctx, hx(rec["m"]), 0)
    for case in ("priv_f32_p7", "priv_f64_none", "priv_edge_p7_noobf"):
        enc, dec = golden["encrypt"][case], golden["decrypt"][case]
        ms = dec["m"][len(dec["m"]) - len(enc["raw"]):]
        from xfl_amd.paillier.encoder import int_to_float_gmpy
        for m, e, want in zip(ms, enc["exp"], dec["origin_f64"]):
            v = PaillierEncoder.decode_single(ctx, hx(m), e)
            assert (v if isinstance(v, float) else int_to_float_gmpy(v)).hex() == want


def test_encode_single_and_exponent(golden):
    from xfl_amd.paillier import PaillierContext, PaillierEncoder
    k = golden["key"]
    ctx = PaillierContext().init(n=hx(k["n"]))
    c = golden["encrypt"]["priv_f64_none"]
    for x, e in zip(c["input"], c["exp"]):
        assert PaillierEncoder.cal_exponent(fl(x), None) == e
    assert PaillierEncoder.cal_exponent(1.0, 7) == -24
    assert PaillierEncoder.cal_exponent(np.int32(5), None) == 0
    assert PaillierEncoder.encode_single(ctx, 0.5 * 2 ** -24, -24) == 0
    assert PaillierEncoder.encode_single(ctx, 1.5 * 2 ** -24, -24) == 2
    assert PaillierEncoder.encode_single(ctx, -1.0, 0) == ctx.n - 1


def test_wire_decode_reference_pickle():
    from xfl_amd import compat
    g = load_fixture(FIXTURES[0])
    arr = compat.loads(bytes.fromhex(g["ops"]["wire_a4"]))
    assert [int(r.value) for r in arr] == [hx(v) for v in g["ops"]["a"]["raw"][:4]]
    assert [r.exp for r in arr] == g["ops"]["a"]["exp"][:4]
    data = compat.dumps(arr)
    assert b"common.crypto.paillier.paillier" in data and b"RawCiphertext" in data
    back = compat.loads(compat.decompress(compat.compress(data)))
    assert [int(r.value) for r in back] == [int(r.value) for r in arr]
    assert compat.gmpy2_from_binary(bytes.fromhex("0102701101")) == -70000


def test_keygen_helpers():
    import math
    import random
    from xfl_amd.paillier.utils import get_core_num, getprimeover, invert, is_probable_prime, next_prime
    rng = random.Random(1)
    p = getprimeover(256, rng=rng)
    assert p.bit_length() == 256 and is_probable_prime(p, rng=rng)
    assert next_prime(13) == 17 and next_prime(1) == 2
    assert invert(3, 7) == 5
    with pytest.raises(ZeroDivisionError):
        invert(6, 9)
    assert get_core_num(-1) >= 1 and get_core_num(0) == 1
    assert math.gcd(p, 2) == 1


def test_device_key_bits():
    from xfl_amd.paillier.context import device_key_bits
    assert device_key_bits((1 << 2047) + 1) == 2048
    assert device_key_bits((1 << 3071) + 1) == 3072
    with pytest.raises(NotImplementedError):
        device_key_bits(15)


def test_utils_scalar_helpers_match_reference_formulas(golden):
    """utils.py:38-76 scalar helpers (API completeness) on the fixture key."""
    from xfl_amd.paillier import utils as U
    k = golden["key"]
    p, q = hx(k["p"]), hx(k["q"])
    n = p * q
    qi = pow(q, -1, p)
    for x in (0, 1, 12345, n - 1, n // 3):
        assert U.crt(x % p, x % q, p, q, qi, n) == x
    assert U.mulmod(n - 1, n - 2, n) == 2
    assert U.powmod(1, n, 7) == 1 and U.powmod(3, 5, 7) == 5
    assert U.invert(3, 7) == 5
    import pytest
    with pytest.raises(ZeroDivisionError):
        U.invert(p, n)
