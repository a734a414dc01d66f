"""PaillierArray: the np.ndarray[object] that Paillier.encrypt returns, with
the element-wise operators, np.sum and np.matmul routed to batched GPU
kernels instead of one Python call per element.

It is an ndarray subclass, so every reference call site that checks
`isinstance(x, np.ndarray)`, indexes, reshapes or concatenates keeps working;
results are bit-identical to the reference's per-element folds (the
homomorphic sum Prod c_i^(2^(e_i - e_min)) is order-free).
Anything not recognised falls back to numpy's per-element object loop, which
calls PaillierCiphertext's own operators (also on the GPU).
"""
import numbers

import numpy as np

from . import ops


def _is_num(x):
    return isinstance(x, (int, float)) and not isinstance(x, bool) or isinstance(x, bool)


def _ct_type():
    from .paillier import PaillierCiphertext
    return PaillierCiphertext


def _raws(cts):
    from .paillier import raws_of
    return raws_of(cts)


class PaillierArray(np.ndarray):
    def __new__(cls, obj):
        return np.asarray(obj, dtype=object).view(cls)

    def __array_finalize__(self, obj):
        pass

    # ------------------------------------------------------------ ufuncs
    def __array_ufunc__(self, ufunc, method, *inputs, out=None, **kwargs):
        if method == "__call__" and out is None and not kwargs:
            try:
                if ufunc is np.add:
                    return _add(*inputs)
                if ufunc is np.subtract:
                    return _sub(*inputs)
                if ufunc is np.multiply:
                    return _mul(*inputs)
                if ufunc is np.true_divide:
                    return _div(*inputs)
                if ufunc is np.matmul:
                    return _matmul(*inputs)
            except _Fallback:
                pass
        args = [np.asarray(x).view(np.ndarray) if isinstance(x, PaillierArray) else x for x in inputs]
        if out is not None:
            out = tuple(np.asarray(o).view(np.ndarray) if isinstance(o, PaillierArray) else o for o in out)
            kwargs["out"] = out
        res = getattr(ufunc, method)(*args, **kwargs)
        return _wrap(res)

    def sum(self, axis=None, dtype=None, out=None, keepdims=False, **kw):
        if axis is None and out is None and not keepdims and not kw and dtype is None:
            flat = np.asarray(self).reshape(-1)
            CT = _ct_type()
            if flat.size >= 2 and all(isinstance(c, CT) for c in flat):
                _check_same_key(list(flat))
                ctx = flat[0].context
                r, e = ops.segment_sums(ctx, _raws(list(flat)), [c.exponent for c in flat],
                                        [0, flat.size])
                return CT(ctx, r[0], int(e[0]))
        return _wrap(np.ndarray.sum(np.asarray(self).view(np.ndarray), axis=axis, dtype=dtype, out=out,
                                    keepdims=keepdims, **kw))


class _Fallback(Exception):
    pass


def _wrap(res):
    if isinstance(res, np.ndarray) and res.dtype == object and not isinstance(res, PaillierArray):
        return res.view(PaillierArray)
    return res


def _obj(x):
    return np.asarray(x, dtype=object) if not isinstance(x, np.ndarray) or x.dtype == object else x.astype(object)


def _check_same_key(cts):
    seen = {}
    first = cts[0].context
    for c in cts:
        k = id(c.context)
        if k in seen:
            continue
        seen[k] = True
        if c.context is not first and c.context.to_public() != first.to_public():
            raise ValueError("Adding two ciphertext with different keys.")


def _add(a, b):
    """element-wise a + b with the reference's semantics (paillier.py:88-126)."""
    CT = _ct_type()
    A, B = np.broadcast_arrays(_obj(a), _obj(b))
    shape = A.shape
    A, B = A.reshape(-1), B.reshape(-1)
    n = A.size
    out = np.empty(n, dtype=object)
    pairs, scal = [], []
    for i in range(n):
        x, y = A[i], B[i]
        xc, yc = isinstance(x, CT), isinstance(y, CT)
        if xc and yc:
            pairs.append((i, x, y))
        elif xc or yc:
            c, s = (x, y) if xc else (y, x)
            if not isinstance(s, (int, float)):
                raise TypeError(f"Adding data of type {type(s)} not supported.")
            scal.append((i, c, s))
        else:
            raise _Fallback()
    if pairs:
        _check_same_key([p[1] for p in pairs] + [p[2] for p in pairs])
        ctx = pairs[0][1].context
        r, e = ops.add(ctx, _raws([p[1] for p in pairs]), [p[1].exponent for p in pairs],
                       _raws([p[2] for p in pairs]), [p[2].exponent for p in pairs])
        for (i, x, _), rv, ev in zip(pairs, r, e):
            out[i] = CT(x.context, rv, int(ev))
    if scal:
        from .paillier import Paillier
        ctx = scal[0][1].context
        enc = Paillier.encrypt(ctx, np.array([s for _, _, s in scal], dtype=object), precision=None,
                               max_exponent=None, obfuscation=False)
        r, e = ops.add(ctx, _raws([c for _, c, _ in scal]), [c.exponent for _, c, _ in scal],
                       [c.raw_ciphertext for c in enc], [c.exponent for c in enc])
        for (i, c, _), rv, ev in zip(scal, r, e):
            out[i] = CT(c.context, rv, int(ev))
    return out.reshape(shape).view(PaillierArray)


def _mul(a, b):
    """element-wise ciphertext * scalar (paillier.py:134-148)."""
    from .encoder import PaillierEncoder
    CT = _ct_type()
    A, B = np.broadcast_arrays(_obj(a), _obj(b))
    shape = A.shape
    A, B = A.reshape(-1), B.reshape(-1)
    n = A.size
    out = np.empty(n, dtype=object)
    items = []
    for i in range(n):
        x, y = A[i], B[i]
        xc, yc = isinstance(x, CT), isinstance(y, CT)
        if xc and yc:
            raise TypeError("Cannot multiply one ciphertext with another ciphertext, try multiply a scalar.")
        if not (xc or yc):
            raise _Fallback()
        c, s = (x, y) if xc else (y, x)
        items.append((i, c, s))
    if items:
        ctx = items[0][1].context
        ks, es = [], []
        for _, c, s in items:
            e = PaillierEncoder.cal_exponent(s, precision=None)
            ks.append(int(PaillierEncoder.encode_single(c.context, s, e)))
            es.append(int(e))
        r = ops.raw_mul(ctx, _raws([c for _, c, _ in items]), ks)
        for (i, c, _), rv, ev in zip(items, r, es):
            out[i] = CT(c.context, rv, ev + c.exponent)
    return out.reshape(shape).view(PaillierArray)


def _neg_each(x):
    return _mul(x, -1) if _has_ct(x) else np.negative(_obj(x))


def _has_ct(x):
    CT = _ct_type()
    return any(isinstance(v, CT) for v in np.asarray(x, dtype=object).reshape(-1))


def _sub(a, b):
    # a - b = a + b*(-1)  (paillier.py:128-132: scalar - ct = (-1)*ct + scalar)
    if _has_ct(b):
        return _add(a, _mul(b, -1))
    return _add(a, np.negative(_obj(b)))


def _div(a, b):
    if _has_ct(b):
        raise _Fallback()
    B = _obj(b)
    return _mul(a, np.vectorize(lambda s: 1 / s, otypes=[object])(B))


def _encode_scalars_vec(X):
    """Vectorised PaillierEncoder.cal_exponent(precision=None) + encode_single
    (encoder.py:29-54) of a plain numeric matrix, as (|k|, k negative, e):
    floats give e = frexp exponent - 53 and |k| = |mantissa| * 2^53 (exact),
    ints e = 0 and |k| = |x|; a negative value encodes to n - |k|, which is
    >= min_value_for_negative for every |k| < 2^63 (the _raw_mul negative
    branch, paillier.py:178-184). None outside the domain where that holds
    without the reference's range errors (non-finite, |x| >= 2^53, |x| below
    2^-960): the caller then runs the scalar encoder element by element."""
    if X.dtype.kind == "f":
        x = X.astype(np.float64)
        ax = np.abs(x)
        if not np.all(np.isfinite(x)) or np.any(ax >= 2.0 ** 53) or np.any((ax < 2.0 ** -960) & (ax != 0)):
            return None
        mant, expo = np.frexp(x)
        kabs = (np.abs(mant) * 2.0 ** 53).astype(np.int64)
        return kabs, x < 0, expo.astype(np.int64) - 53
    if X.dtype.kind in "iu" and X.dtype.itemsize <= 8:
        if X.dtype.kind == "u" and X.size and int(X.max()) >= 2 ** 63:
            return None
        x = X.astype(np.int64)
        if X.dtype.kind == "i" and np.any(x == np.iinfo(np.int64).min):
            return None
        return np.abs(x), x < 0, np.zeros(X.shape, dtype=np.int64)
    return None


def _matmul(a, b):
    """enc[B] @ X[B, D] (logistic_regression/trainer.py:166): per output j,
    Prod_i base_i^(k'_ij * 2^(d_ij)) with base_i = c_i or c_i^-1 (negative
    scalars), d_ij aligning e_i + e_kij to the column minimum; = the
    reference's object-dtype dot product bit for bit."""
    from .encoder import PaillierEncoder
    CT = _ct_type()
    A = np.asarray(a, dtype=object)
    X = np.asarray(b)
    if A.ndim != 1 or X.ndim != 2 or X.dtype == object or A.shape[0] != X.shape[0] or A.shape[0] == 0:
        raise _Fallback()
    if not all(isinstance(c, CT) for c in A):
        raise _Fallback()
    _check_same_key(list(A))
    ctx = A[0].context
    Bn, D = X.shape
    cexp = np.array([c.exponent for c in A], dtype=np.int64)
    vec = _encode_scalars_vec(X)
    if vec is not None:
        kabs, neg_a, e_a = vec
        ks = kabs.tolist()
        neg = neg_a.tolist()
        ex = cexp[:, None] + e_a
    else:
        thr = ctx.min_value_for_negative
        ks = [[0] * D for _ in range(Bn)]
        neg = [[False] * D for _ in range(Bn)]
        ex = np.zeros((Bn, D), dtype=np.int64)
        for i in range(Bn):
            for j in range(D):
                s = X[i, j].item()
                e = PaillierEncoder.cal_exponent(s, precision=None)
                k = int(PaillierEncoder.encode_single(ctx, s, e))
                if k >= thr:
                    ks[i][j], neg[i][j] = ctx.n - k, True
                else:
                    ks[i][j] = k
                ex[i, j] = cexp[i] + e
    emin = ex.min(axis=0)
    need_inv = [i for i in range(Bn) if any(neg[i])]
    # bases: the B ciphertexts, then the inverses of those with a negative scalar
    bases = _raws(list(A))
    inv_slot = {}
    if need_inv:
        r = ops.powmod(ctx, [bases[i] for i in need_inv], [1] * len(need_inv), invert_first=True)
        for i, v in zip(need_inv, r):
            inv_slot[i] = len(bases)
            bases.append(v)
    idx = [[inv_slot[i] if neg[i][j] else i for i in range(Bn)] for j in range(D)]
    exps = [[ks[i][j] << int(ex[i, j] - emin[j]) for i in range(Bn)] for j in range(D)]
    r = ops.multiexp(ctx, bases, idx, exps)
    out = np.empty(D, dtype=object)
    for j in range(D):
        out[j] = CT(ctx, r[j], int(emin[j]))
    return out.view(PaillierArray)
