"""Paillier.serialize of device-resident arrays through the pipeline
(wire.encode_device: bit lengths on the device -> layout -> chunked D2H copies
overlapping the host encode, paillier.py:244-258): the bytes equal the
two-step path (download, then the native pickle encoder + the zstd raw
frame), with and without compression, for arrays of several chunk counts,
slices and odd sizes, and for the asynchronous encryption that feeds it
(resident.encrypt_floats returns before its kernels finish). The payloads
decode back with the reference-format decoder."""
import numpy as np
import pytest

from tests.conftest import hx, load_fixture

pytestmark = pytest.mark.gpu


def _ctx(fx="paillier_2048_djn.json"):
    from xfl_amd.paillier import PaillierContext
    k = load_fixture(fx)["key"]
    return PaillierContext().init(hx(k["p"]), hx(k["q"]), djn_h_pow_n=hx(k["h_pow_n"]) if k["djn_on"] else None)


@pytest.mark.parametrize("fx", ["paillier_2048_djn.json", "paillier_3072_djn.json"])
def test_pipeline_bytes_equal_two_step(fx):
    from xfl_amd import compat
    from xfl_amd.paillier import Paillier
    from xfl_amd.paillier import wire
    ctx = _ctx(fx)
    rng = np.random.default_rng(4)
    for n in (wire.PIPE_MIN, 3 * wire.PIPE_CHUNK + 12345):
        x = rng.standard_normal(n).astype(np.float32)
        for comp in (False, True):
            enc = Paillier.encrypt(ctx, x, precision=7)
            assert enc.is_resident and enc._st.h is None
            got = Paillier.serialize(enc, compression=comp)  # the pipeline (words only in HBM)
            assert enc._st.h is None
            want = wire.encode_words(enc.words, enc.exponents, enc.shape)
            if comp:
                want = compat.compress(want)
            assert got == want, (n, comp)
            back = Paillier.ciphertext_from(ctx, got, compression=comp)
            assert np.array_equal(back.words, enc.words) and np.array_equal(back.exponents, enc.exponents)
    # a slice of a resident array (a view into the device words), and a 2-D shape
    enc = Paillier.encrypt(ctx, rng.standard_normal(200000).astype(np.float32), precision=7)
    view = enc[1000:1000 + 131072]
    got = Paillier.serialize(view)
    assert got == compat.compress(wire.encode_words(view.words, view.exponents, view.shape))
    m = Paillier.encrypt(ctx, rng.standard_normal((300, 400)), precision=None)
    got = Paillier.serialize(m, compression=False)
    assert got == wire.encode_words(m.words, m.exponents, m.shape)
    assert Paillier.ciphertext_from(ctx, got, compression=False).shape == (300, 400)


def test_async_encrypt_raises_and_decrypts():
    from xfl_amd.paillier import Paillier
    ctx = _ctx()
    x = np.random.default_rng(5).standard_normal(100000)
    enc = Paillier.encrypt(ctx, x, precision=7)
    assert np.allclose(Paillier.decrypt(ctx, enc), x.astype(np.float32), atol=1e-6)
    bad = x.copy()
    bad[77777] = np.inf
    with pytest.raises(OverflowError):
        Paillier.encrypt(ctx, bad, precision=7)
    bad[77777] = np.nan
    with pytest.raises(ValueError):
        Paillier.encrypt(ctx, bad, precision=7)


def test_pipeline_over_running_encryption_and_in_place_writes():
    """An encryption launched in ENC_SUB-row pieces on two streams (each
    marked by an event) serializes while it runs - the copy stream waits per
    chunk only for the launches that write its rows - and the bytes equal the
    two-step path; rows rewritten in place afterwards (an obfuscated view,
    resident.put_rows) drop the marks, so the next serialize sees them."""
    from xfl_amd.paillier import Paillier
    from xfl_amd.paillier import wire
    ctx = _ctx()
    rng = np.random.default_rng(6)
    n = 2 * wire.ENC_SUB + 3 * wire.PIPE_CHUNK + 77
    x = rng.standard_normal(n).astype(np.float32)
    enc = Paillier.encrypt(ctx, x, precision=7)
    assert len(enc._st.d._xhe_ready) == -(-n // wire.ENC_SUB) and enc._st.d._xhe_bits.shape == (n,)
    from xfl_amd import _native as nat
    copies = nat.shrink_copies
    got = Paillier.serialize(enc, compression=True)
    assert nat.shrink_copies == copies  # the payload was cut in place
    assert got == wire.encode_words(enc.words, enc.exponents, enc.shape, compression=True)
    enc2 = Paillier.encrypt(ctx, x, precision=7)
    Paillier.obfuscate(enc2[1000:2000])
    assert not hasattr(enc2._st.d, "_xhe_ready") and not hasattr(enc2._st.d, "_xhe_bits")
    enc2._st.h = None
    got2 = Paillier.serialize(enc2, compression=False)
    assert got2 == wire.encode_words(enc2.words, enc2.exponents, enc2.shape)
    assert np.allclose(Paillier.decrypt(ctx, enc2), x, atol=1e-6)
