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


def test_host_encrypt_chunking_is_invisible():
    """xhe_encrypt_f64_host pipelines 256k-element chunks (per-slot streams,
    pinned staging); the
    randomness is drawn at global element positions, so the result equals one
    device-resident encode + draw + encrypt of the whole batch, and spot
    elements equal the oracle's encryption with the drawn a."""
    import ctypes

    import torch

    from xfl_amd import _native as nat
    g = load_fixture(FIXTURES[0])
    dk = _dkey(g)
    ok = _okey(g)
    L = nat.lib()
    n = 600_003  # three chunks, the last one ragged
    x = np.random.default_rng(3).standard_normal(n)
    seed, nonce = bytes(range(32)), 77
    vp = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    ct = np.empty((n, dk.n2w), np.uint32)
    ex = np.empty(n, np.int32)
    st = np.empty(n, np.int32)
    nat.check(L.xhe_encrypt_f64_host(dk.handle, vp(x), n, 7, 0, 0, 1, seed, nonce, vp(ct), vp(ex), vp(st)), "host")
    xd = torch.from_numpy(x).cuda()
    m = torch.empty((n, dk.nw), dtype=torch.int32, device="cuda")
    e = torch.empty(n, dtype=torch.int32, device="cuda")
    s = torch.empty(n, dtype=torch.int32, device="cuda")
    r = torch.empty((n, dk.rand_words), dtype=torch.int32, device="cuda")
    c = torch.empty((n, dk.n2w), dtype=torch.int32, device="cuda")
    strm = torch.cuda.current_stream().cuda_stream
    nat.check(L.xhe_encode_f64(dk.handle, xd.data_ptr(), n, 7, 0, 0, m.data_ptr(), e.data_ptr(), s.data_ptr(), strm))
    nat.check(L.xhe_rand(dk.handle, seed, nonce, n, r.data_ptr(), None, strm))
    nat.check(L.xhe_encrypt(dk.handle, m.data_ptr(), r.data_ptr(), n, c.data_ptr(), strm))
    torch.cuda.synchronize()
    assert np.array_equal(c.cpu().numpy().view(np.uint32), ct)
    assert np.array_equal(e.cpu().numpy(), ex) and not st.any()
    for i in (0, 262143, 262144, 524288, n - 1):
        mi = O.encode_element(ok, float(x[i]), 7)[0]
        ai = nat.words_to_ints(r[i].cpu().numpy().view(np.uint32))
        assert nat.words_to_ints(ct[i]) == O.encrypt_m(ok, mi, ai)


@pytest.mark.parametrize("fx", FIXTURES)
@pytest.mark.parametrize("count", [1, 300, 1024, 1100, 5000, 20000, 30000])
def test_decrypt_shapes_bit_exact(fx, count):
    """The decrypt exponentiation runs in four lane shapes chosen by batch
    size (2048-bit keys: a block per residue in RNS form up to 1,024 elements, then
    16 lanes per residue up to 5,120, 4 up to 28,672, then 1): the golden
    ciphertexts tiled to each regime decrypt to the golden m."""
    from xfl_amd._native import ints_to_words, words_to_ints
    g = load_fixture(fx)
    dk = _dkey(g)
    raws, ms = [], []
    for case in ("priv_f32_p7", "priv_packed_p0", "pub_i32_none"):
        enc, dec = g["encrypt"][case], g["decrypt"][case]
        raws += [hx(r) for r in enc["raw"]]
        ms += [hx(m) for m in dec["m"][len(dec["m"]) - len(enc["raw"]):]]
    reps = -(-count // len(raws))
    cw = ints_to_words((raws * reps)[:count], dk.n2w)
    out = words_to_ints(dk.decrypt_words(cw))
    assert out == (ms * reps)[:count]


@pytest.mark.parametrize("count", [7, 300, 700, 1500])
def test_decrypt_arbitrary_residues(count):
    """Any c < n^2 coprime to n (as every ciphertext is), not only
    well-formed ciphertexts, decrypts as the reference's arithmetic does
    (paillier.py:341-368, restated by oracle.decrypt_raw): edge residues (1,
    n^2 - 1, next to p^2 and q^2) and random ones, in the small-batch
    (whole-wave) and the 16-lane shapes."""
    import random

    from xfl_amd._native import ints_to_words, words_to_ints
    g = load_fixture("paillier_2048_djn.json")
    dk = _dkey(g)
    ok = _okey(g)
    p, q, n = hx(g["key"]["p"]), hx(g["key"]["q"]), hx(g["key"]["n"])
    n2 = n * n
    rnd = random.Random(count)
    edge = [1, n2 - 1, p * p - 1, p * p + 1, q * q - 2, q * q + 3, n + 1, p * q * q + 5]
    cs = (edge + [rnd.randrange(1, n2) for _ in range(count)])[:count]
    out = words_to_ints(dk.decrypt_words(ints_to_words(cs, dk.n2w)))
    assert out == [O.decrypt_raw(ok, c) for c in cs]
