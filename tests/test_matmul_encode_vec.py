"""CPU: the vectorised scalar encoding used by the encrypted matmul
(array._encode_scalars_vec) equals PaillierEncoder.cal_exponent(precision=None)
+ encode_single (encoder.py:29-54) element by element, including the
negative-scalar split of PaillierCiphertext._raw_mul (paillier.py:178-184),
and declines inputs outside its domain."""
import numpy as np
import pytest

from tests.conftest import FIXTURES, hx, load_fixture


def _ctx():
    from xfl_amd.paillier import PaillierContext
    k = load_fixture(FIXTURES[0])["key"]
    return PaillierContext().init(hx(k["p"]), hx(k["q"]))


def _scalar(ctx, X):
    from xfl_amd.paillier.encoder import PaillierEncoder
    out = []
    for s in X.reshape(-1):
        v = s.item()
        e = PaillierEncoder.cal_exponent(v, precision=None)
        k = int(PaillierEncoder.encode_single(ctx, v, e))
        neg = k >= ctx.min_value_for_negative
        out.append((ctx.n - k if neg else k, neg, e))
    return out


@pytest.mark.parametrize("dtype", [np.float32, np.float64, np.int32, np.int64, np.int16, np.uint32])
def test_vectorised_encoding_matches_scalar(dtype):
    from xfl_amd.paillier.array import _encode_scalars_vec
    ctx = _ctx()
    rng = np.random.default_rng(5)
    if np.dtype(dtype).kind == "f":
        X = np.concatenate([rng.standard_normal(200) * 10.0 ** rng.integers(-30, 12, 200),
                            [0.0, -0.0, 1.0, -1.0, 0.5, 2.0 ** -900, -(2.0 ** 52), 3.0e-38]]).astype(dtype)
    else:
        info = np.iinfo(dtype)
        X = np.concatenate([rng.integers(max(info.min, -2 ** 40), min(info.max, 2 ** 40), 200),
                            [0, 1, info.max, info.min + 1 if info.min < 0 else 0]]).astype(dtype)
    X = X.reshape(-1, 4)
    kabs, neg, e = _encode_scalars_vec(X)
    got = list(zip(kabs.reshape(-1).tolist(), neg.reshape(-1).tolist(), e.reshape(-1).tolist()))
    assert got == _scalar(ctx, X)


@pytest.mark.parametrize("bad", [np.inf, -np.inf, np.nan, 2.0 ** 53, 2.0 ** -1000])
def test_vectorised_encoding_declines_outside_domain(bad):
    from xfl_amd.paillier.array import _encode_scalars_vec
    X = np.array([[1.0, bad]], dtype=np.float64)
    assert _encode_scalars_vec(X) is None


def test_vectorised_encoding_declines_int64_min():
    from xfl_amd.paillier.array import _encode_scalars_vec
    assert _encode_scalars_vec(np.array([[np.iinfo(np.int64).min, 1]], dtype=np.int64)) is None
