"""Device-resident PaillierArray (xfl_amd/paillier/resident.py): results of
batched operations stay in HBM and chain without PCIe round trips; the host
copy appears only on host access. Every result is compared bit for bit with
the host-buffer path ($XHE_RESIDENT=0) on the same inputs, and that path is
pinned to the reference's golden vectors by tests/test_gpu_dropin.py."""
import numpy as np
import pytest

from tests import dropin_cases as C
from tests.conftest import load_fixture

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def keys():
    return C.ctxs(load_fixture("paillier_2048_djn.json"))


def _host_mode(monkeypatch, on):
    if on:
        monkeypatch.setenv("XHE_RESIDENT", "0")
    else:
        monkeypatch.delenv("XHE_RESIDENT", raising=False)


def _words(a):
    return np.asarray(a.words).copy(), a.exponents.copy()


def test_chain_stays_in_hbm(keys):
    """encrypt -> + -> * -> sum -> matmul -> decrypt: no host copy is made of
    any intermediate, and the decrypted values are the plaintext results"""
    from xfl_amd.paillier import Paillier
    priv, _ = keys
    rng = np.random.default_rng(3)
    x = (rng.random(4096) * 20 - 10).astype(np.float32)
    y = (rng.random(4096) * 20 - 10).astype(np.float32)
    cx, cy = Paillier.encrypt(priv, x, precision=7), Paillier.encrypt(priv, y, precision=7)
    assert cx.is_resident and cx._st.h is None
    s = cx + cy
    m = s * 0.5
    assert s.is_resident and m.is_resident and s._st.h is None and m._st.h is None
    assert np.all(np.abs(Paillier.decrypt(priv, m) - (x + y) * 0.5) < 1e-3)
    X = rng.random((4096, 3))
    mv = cx @ X
    assert mv.is_resident and cx._st.h is None
    assert np.allclose(Paillier.decrypt(priv, mv), x.astype(np.float64) @ X, atol=1e-2)
    tot = np.sum(cx.reshape(64, 64), axis=1)
    assert tot.is_resident
    assert np.allclose(Paillier.decrypt(priv, tot), x.astype(np.float64).reshape(64, 64).sum(axis=1), atol=1e-3)
    assert cx._st.h is None  # nothing above needed the words on the host


def test_resident_equals_host_path(keys, monkeypatch):
    """deterministic encryptions and every batched op: identical words and
    exponents in both modes (mixed exponents, negative scalars, inversions)"""
    from xfl_amd.paillier import Paillier
    priv, pub = keys
    rng = np.random.default_rng(5)
    x = rng.standard_normal(300) * 100
    k = rng.standard_normal(300)
    X = rng.standard_normal((300, 4))
    res = {}
    for host in (True, False):
        _host_mode(monkeypatch, host)
        a = Paillier.encrypt(pub, x, precision=None, obfuscation=False)
        b = Paillier.encrypt(pub, x[::-1].copy(), precision=7, obfuscation=False)
        assert a.is_resident != host
        outs = [a, b, a + b, a - b, a * k, b * -3, a / 7.0, 2.5 - a, a @ X, X.T @ b, np.sum(a.reshape(20, 15), axis=0),
                np.concatenate([a[:10], b[5:9]]), a.reshape(15, 20).T, a[[3, 3, 1]]]
        res[host] = [_words(o) for o in outs]
        res[host].append(_words(Paillier.encrypt(pub, np.arange(-5, 5), obfuscation=False)))
    _host_mode(monkeypatch, False)
    for i, (h, d) in enumerate(zip(res[True], res[False])):
        assert np.array_equal(h[0], d[0]) and np.array_equal(h[1], d[1]), i


def test_views_assignment_and_obfuscate(keys):
    """slices share the storage; assignment goes to the host copy and drops
    the stale device copy; obfuscating a view re-randomises only its rows"""
    from xfl_amd.paillier import Paillier
    priv, _ = keys
    x = np.arange(16, dtype=np.float64) - 8
    c = Paillier.encrypt(priv, x, precision=7)
    v = c[2:6]
    v[0] = c[9]
    assert c[2].raw_ciphertext == c[9].raw_ciphertext
    assert not c.is_resident  # the host copy was written
    want = x.copy()
    want[2] = x[9]
    assert np.allclose(Paillier.decrypt(priv, c + c), 2 * want, atol=1e-5)
    c.to_device()
    before = np.asarray(c.words).copy()
    c._st.h = None
    Paillier.obfuscate(c[4:8])
    after = np.asarray(c.words)
    assert np.array_equal(before[:4], after[:4]) and np.array_equal(before[8:], after[8:])
    assert not np.any(np.all(before[4:8] == after[4:8], axis=1))
    assert np.allclose(Paillier.decrypt(priv, c), want, atol=1e-5)


def test_serialize_resident(keys):
    """serialize downloads lazily and writes the same bytes as the host copy"""
    from xfl_amd.paillier import Paillier, PaillierArray
    priv, _ = keys
    c = Paillier.encrypt(priv, np.linspace(-3, 3, 257), precision=7)
    assert c._st.h is None
    wire = Paillier.serialize(c, compression=False)
    host = PaillierArray.from_buffers(priv, np.asarray(c.words).copy(), c.exponents.copy(), c.shape)
    assert wire == Paillier.serialize(host, compression=False)
    back = Paillier.ciphertext_from(priv, wire, compression=False)
    assert not back.is_resident
    assert np.allclose(Paillier.decrypt(priv, back), np.linspace(-3, 3, 257), atol=1e-6)
