"""HIP path vs the reference's golden vectors (bit-exact), through the C ABI."""
import numpy as np
import pytest

from oracle import paillier_oracle as O
from tests.conftest import FIXTURES, hx, load_fixture

pytestmark = pytest.mark.gpu


def _dkey(g, private=True):
    from xfl_amd._native import DeviceKey
    k = g["key"]
    h = hx(k["h_pow_n"]) if k["djn_on"] else None
    if private:
        return DeviceKey(g["key_bits"], hx(k["n"]), hx(k["p"]), hx(k["q"]), h)
    return DeviceKey(g["key_bits"], hx(k["n"]), None, None, h)


def _okey(g):
    k = g["key"]
    return O.derive_private(hx(k["p"]), hx(k["q"]), hx(k["h_pow_n"]) if k["djn_on"] else None)


ENC_CASES = ["priv_f32_p7", "priv_f64_none", "priv_packed_p0", "pub_f32_p7", "pub_f64_none_max-60",
             "pub_i32_none", "priv_edge_p7_noobf"]


@pytest.mark.parametrize("fx", FIXTURES)
@pytest.mark.parametrize("case", ENC_CASES)
def test_encrypt_bit_exact(fx, case):
    """Every encryption mode (DJN/non-DJN x private CRT/public, obfuscated or
    not) with the reference's recorded obfuscation draws."""
    from xfl_amd._native import ints_to_words, words_to_ints
    g = load_fixture(fx)
    c = g["encrypt"][case]
    dk = _dkey(g, private=c["private"])
    ok = _okey(g)
    xs = [hx(v) for v in c["input"]] if c["kind"] == "int" else [float.fromhex(v) for v in c["input"]]
    ms = [O.encode_element(ok, x, c["precision"], c["max_exponent"])[0] for x in xs]
    mw = ints_to_words(ms, dk.nw)
    rw = ints_to_words([hx(r) for r in c["rand"]], dk.rand_words) if c["obfuscation"] else None
    out = words_to_ints(dk.encrypt_words(mw, rw))
    assert out == [hx(r) for r in c["raw"]]


@pytest.mark.parametrize("fx", FIXTURES)
@pytest.mark.parametrize("case", ["priv_f32_p7", "pub_f32_p7", "priv_f64_none", "priv_packed_p0",
                                  "priv_edge_p7_noobf", "pub_i32_none"])
def test_decrypt_bit_exact(fx, case):
    from xfl_amd._native import ints_to_words, words_to_ints
    g = load_fixture(fx)
    dk = _dkey(g)
    enc = g["encrypt"][case]
    dec = g["decrypt"][case]
    ms = dec["m"][len(dec["m"]) - len(enc["raw"]):]
    cw = ints_to_words([hx(r) for r in enc["raw"]], dk.n2w)
    out = words_to_ints(dk.decrypt_words(cw))
    assert out == [hx(m) for m in ms]
