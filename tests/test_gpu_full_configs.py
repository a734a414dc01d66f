"""BASELINE configs 3 and 5 at their full sizes through the drop-in, on the
GPU, checked where a size-independent property or a cheap exact checker
exists:

* config 5 (XGBoost histogram, 100 k samples x 64 features x 256 bins): the
  label side's embed -> Paillier.encrypt(precision=0) -> serialize, the
  trainer's ciphertext_from -> Feature.create (core/tree/big_feature.py:43-46)
  -> groupby(col)['xfl_grad_hess'].agg({'count', 'sum'}) per feature
  (xgboost/decision_tree_trainer.py:151-152) on the pandas ciphertext column
  (PaillierDtype, one segmented product per call). 4 features bit-exact
  against Python-integer products of the same ciphertexts (the oracle's
  sum_ct: exponents are all 0); all 64 decrypt to the exact integer sums of
  the embedded values; counts = bincount.
* config 3 (10 M float32 gradients, precision 7): one full reduction whose
  decrypt equals the exact integer sum of the encodings (mod n, signed), and
  the pairwise c * d of two encrypted vectors on a 4,096-element sample
  against Python's a b mod n^2 plus a decrypt of the whole pairwise sum.
* the golden pandas cases (tests/dropin_cases.xgb_histogram_pandas) with the
  column resident in HBM, at every key size.
"""
import numpy as np
import pytest

from tests import dropin_cases as C
from tests.conftest import FIXTURES, hx, load_fixture

pytestmark = pytest.mark.gpu


def _ctx(fx="paillier_2048_djn.json"):
    from xfl_amd.paillier import PaillierContext
    k = load_fixture(fx)["key"]
    return PaillierContext().init(hx(k["p"]), hx(k["q"]), djn_h_pow_n=hx(k["h_pow_n"]) if k["djn_on"] else None)


@pytest.mark.parametrize("fx", FIXTURES)
def test_xgb_histogram_pandas_resident(fx):
    C.xgb_histogram_pandas(fx, resident=True)


def test_config5_full_size_pandas_groupby():
    import time

    import pandas as pd

    from bench import xgb_inputs
    from xfl_amd import _native as nat
    from xfl_amd.paillier import Paillier
    from xfl_amd.paillier.array import PaillierDtype
    from xfl_amd.paillier_acceleration import embed
    ctx = _ctx()
    pub = ctx.to_public()
    n, nfeat, nbins = 100_000, 64, 256
    g, h, values = xgb_inputs(n, nfeat, nbins)
    ints = embed([g, h], interval=1 << 128, precision=64)
    enc = Paillier.encrypt(ctx, ints, precision=0)
    wire = Paillier.serialize(enc, compression=False)
    grad_hess = Paillier.ciphertext_from(pub, wire, compression=False)
    data = pd.concat([pd.DataFrame(range(n), columns=['xfl_id']), pd.DataFrame(grad_hess, columns=['xfl_grad_hess']),
                      values], axis=1)
    assert isinstance(data['xfl_grad_hess'].dtype, PaillierDtype)
    cols = list(values.columns)
    t0 = time.time()
    res = [data.groupby([c])['xfl_grad_hess'].agg({'count', 'sum'}) for c in cols]
    sums = [r['sum'].to_numpy() for r in res]
    print(f"64 groupby calls + to_numpy (first call uploads the column): {time.time() - t0:.3f} s")
    words = grad_hess.words
    n2 = pub.n_square
    raws = nat.words_to_ints(words)
    for f in range(nfeat):
        b = values[cols[f]].to_numpy()
        assert res[f].index.tolist() == list(range(nbins))
        assert res[f]['count'].tolist() == np.bincount(b, minlength=nbins).tolist()
        if f < 4:  # every bin's residue against Python-integer products
            want = [1] * nbins
            for i in range(n):
                want[b[i]] = want[b[i]] * raws[i] % n2
            assert [c.raw_ciphertext for c in sums[f]] == want, cols[f]
            assert all(c.exponent == 0 for c in sums[f])
    # every feature's bins decrypt to the exact sums of the embedded integers
    allbins = Paillier.decrypt(ctx, np.concatenate(sums), out_origin=True)
    for f in range(nfeat):
        b = values[cols[f]].to_numpy()
        want = [sum(ints[b == k].tolist()) for k in range(nbins)]
        assert [int(v) for v in allbins[f * nbins:(f + 1) * nbins]] == want, cols[f]


def test_config3_full_size_reduction_and_pairwise():
    from xfl_amd import _native as nat
    from xfl_amd.paillier import Paillier
    from xfl_amd.paillier.encoder import PaillierEncoder
    ctx = _ctx()
    n = 10_000_000
    gr = (np.random.default_rng(1).standard_normal(n).astype(np.float32) * np.float32(1e-2))
    c = Paillier.encrypt(ctx, gr, precision=7)
    assert c.is_resident and c.shape == (n,)
    # full reduction: decrypt = the exact sum of the encodings round(x 2^24) (encoder.py:48-54; all exponents -24)
    s = np.sum(c)
    m_exact = int(np.sum(np.round(gr.astype(np.float64) * 2.0 ** 24).astype(np.int64)))
    assert s.exponent == -24
    dec = Paillier.decrypt(ctx, s, out_origin=True)
    assert dec == PaillierEncoder.decode_single(ctx, m_exact % ctx.n, -24)
    # pairwise c * d (paillier.py:153-154) of two encrypted 10 M vectors
    d = Paillier.encrypt(ctx, gr[::-1].copy(), precision=7)
    t = c + d
    assert t.is_resident
    idx = np.unique(np.concatenate([[0, 1, n - 1], np.random.default_rng(5).integers(0, n, 4093)]))
    n2 = ctx.n_square
    ci, di, ti = (nat.words_to_ints(x[idx].words) for x in (c, d, t))
    assert [a * b % n2 for a, b in zip(ci, di)] == ti
    assert t[idx].exponents.tolist() == [-24] * len(idx)
    got = Paillier.decrypt(ctx, t)
    want = (np.round(gr.astype(np.float64) * 2.0 ** 24) + np.round(gr[::-1].astype(np.float64) * 2.0 ** 24)) / 2.0 ** 24
    assert np.array_equal(got, want.astype(np.float32))
