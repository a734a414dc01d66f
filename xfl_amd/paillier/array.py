"""PaillierArray: the ciphertext array Paillier.encrypt / ciphertext_from /
the batched operators return - flat buffers underneath, objects on demand.

The reference hands out np.ndarray(dtype=object) of PaillierCiphertext, one
Python object (and one mpz) per element (paillier.py:289-339). Here an array
is three things: the context, uint32 words [size, n2w] (little-endian
residues mod n^2, C order over `shape`) and int32 exponents [size] - the
layout the kernels, the wire codec (include/xhe.h) and RCCL move - and a
PaillierCiphertext is created only when an element is read. Serialize,
decrypt, +, -, *, /, np.sum, np.matmul and obfuscate run on the buffers
without creating Python ints.

Array protocol: shape / ndim / size / len / iteration / indexing / reshape /
flatten / ravel / transpose / copy / tolist / astype(object), the numpy
operators and ufuncs, np.sum / np.concatenate / np.stack / np.matmul / np.dot
through __array_function__, and __array__ for anything else (pandas columns,
np.asarray, lists of arrays): that materializes the object array the
reference would have held, so every remaining numpy/pandas path computes
exactly what the reference computes (per element, through PaillierCiphertext's
own operators, also on the GPU). Results are bit-identical to the reference's
per-element folds (the homomorphic sum is order-free).

Differences from an object ndarray: basic slices of a 1-D array share the
buffers (like numpy views); other indexing returns copies; elements read
twice are two equal PaillierCiphertext objects, not one; mutate through
arr[i] = ciphertext, not by mutating an element read earlier.

pandas: a PaillierArray is also a pandas ExtensionArray (dtype
`PaillierDtype`, name "paillier", kind 'O'), so a DataFrame column built from
one keeps the flat words instead of one PaillierCiphertext object per row -
`pd.DataFrame(grad_hess, columns=['xfl_grad_hess'])` (core/tree/big_feature.py:
43-46), `data['xfl_grad_hess'] = grad_hess` (core/tree_ray/big_feature.py:74).
XFL's histogram calls then reach the segmented-product kernel once per call:
`groupby(col)['xfl_grad_hess'].agg({'count', 'sum'})`
(xgboost/decision_tree_trainer.py:151-152, core/tree_ray/xgb_actor.py:342-344)
and `groupby(index).sum(numeric_only=False)` (xgb_actor.py:453) go through
`_groupby_op`, `Series.sum` through `_reduce`, concat / loc / iloc / merge
through `_concat_same_type` / `take`. Results equal pandas' object-dtype left
folds bit for bit (the same per-group row order, `ops.fold_gap_powers`).
Missing entries (an outer merge's reindex) are NaN on read; `fillna(0)`
stores the unobfuscated encryption of 0 (raw 1, exponent 0), which adds
exactly as the reference's int 0 cell does (paillier.py:93-102). Other
groupby reductions fall back to pandas' per-group Python path over the
PaillierCiphertext objects (the reference's semantics).
"""
import numbers

import numpy as np

from .. import _native as nat
from . import ops, resident
from .resident import Rows

try:  # pandas is what XFL's tree operators use; without it PaillierArray is a plain class
    from pandas.api.extensions import ExtensionArray as _EABase
    from pandas.api.extensions import ExtensionDtype as _EADtypeBase
    from pandas.api.extensions import register_extension_dtype as _register_dtype
except ImportError:  # pragma: no cover - pandas is in the image
    _EABase, _EADtypeBase = object, object

    def _register_dtype(cls):
        return cls

# exponent of a missing (NA) entry: no encoder produces it (|e| < 2^31 - 1)
NA_EXP = np.iinfo(np.int32).min


def _ct_type():
    from .paillier import PaillierCiphertext
    return PaillierCiphertext


@_register_dtype
class PaillierDtype(_EADtypeBase):
    """pandas dtype of a PaillierArray column: scalars are PaillierCiphertext,
    missing values NaN. Not numeric (pandas' numeric_only reductions skip it,
    as they skip the reference's object columns)."""
    name = "paillier"
    kind = "O"
    na_value = np.nan
    _is_numeric = False
    _metadata = ()

    @property
    def type(self):
        return _ct_type()

    @classmethod
    def construct_array_type(cls):
        return PaillierArray

    @classmethod
    def construct_from_string(cls, string):
        if not isinstance(string, str):
            raise TypeError(f"'construct_from_string' expects a string, got {type(string)}")
        if string == cls.name:
            return cls()
        raise TypeError(f"Cannot construct a 'PaillierDtype' from '{string}'")

    def __repr__(self):
        return "PaillierDtype()"


def _same_key(c1, c2):
    return c1 is c2 or c1 is None or c2 is None or c1.to_public() == c2.to_public()


class _Fallback(Exception):
    pass


class PaillierArray(_EABase):
    __array_priority__ = 1000

    # ------------------------------------------------------------ construction
    def __init__(self, obj, context=None):
        """PaillierArray(ciphertexts): from an object array / nested list of
        PaillierCiphertext (one key), or another PaillierArray (copy)."""
        if isinstance(obj, PaillierArray):
            c = obj.copy()
            self._set(c.context, c._st, c._lo, c._e, c._shape)
            return
        arr = np.asarray(obj, dtype=object)
        flat = arr.reshape(-1)
        CT = _ct_type()
        for c in flat:
            if not isinstance(c, CT):
                raise TypeError(f"PaillierArray holds PaillierCiphertext elements, got {type(c)}")
        ctx = context
        if ctx is None:
            for c in flat:
                if c.context is not None:
                    ctx = c.context
                    break
        for c in flat:
            if not _same_key(c.context, ctx):
                raise ValueError("Adding two ciphertext with different keys.")
        from .paillier import raws_of
        raws = raws_of(list(flat))
        n2w = _n2w(ctx, raws)
        w = nat.ints_to_words(raws, n2w) if raws else np.zeros((0, n2w), dtype=np.uint32)
        e = np.fromiter((c.exponent for c in flat), dtype=np.int32, count=flat.size)
        self._set(ctx, Rows(h=np.ascontiguousarray(w)), 0, e, arr.shape)

    @classmethod
    def from_buffers(cls, context, words, exps, shape=None):
        """Wrap flat host buffers (no copy when already uint32/int32 C-contiguous)."""
        self = cls.__new__(cls)
        words = np.ascontiguousarray(words, dtype=np.uint32)
        exps = np.ascontiguousarray(exps, dtype=np.int32).reshape(-1)
        if shape is None:
            shape = (exps.shape[0],)
        if words.ndim != 2:
            words = words.reshape(exps.shape[0], -1) if exps.shape[0] else np.zeros((0, 1), dtype=np.uint32)
        self._set(context, Rows(h=words), 0, exps, tuple(int(s) for s in shape))
        return self

    @classmethod
    def from_device(cls, context, dwords, exps, shape=None):
        """Wrap device words (an int32 tensor [size, n2w] in HBM, resident.py)
        and host exponents; the host copy is made on first host access."""
        self = cls.__new__(cls)
        exps = np.ascontiguousarray(exps, dtype=np.int32).reshape(-1)
        if shape is None:
            shape = (exps.shape[0],)
        self._set(context, Rows(d=dwords), 0, exps, tuple(int(s) for s in shape))
        return self

    def _set(self, ctx, st, lo, e, shape):
        shape = tuple(shape)
        if int(np.prod(shape, dtype=np.int64)) != e.shape[0] or st.count < lo + e.shape[0]:
            raise ValueError(f"PaillierArray: {st.count - lo} rows / {e.shape[0]} exponents for shape {shape}")
        self.context = ctx
        self._st = st   # word storage, shared with views (resident.Rows)
        self._lo = lo   # first row of this array in it
        self._e = e
        self._shape = shape

    def _view(self, lo, e, shape):
        """an array over rows [self._lo + lo, ...) of the same storage"""
        v = PaillierArray.__new__(PaillierArray)
        v._set(self.context, self._st, self._lo + lo, e, shape)
        return v

    def _whole(self):
        return self._lo == 0 and self.size == self._st.count

    # ------------------------------------------------------------ buffers
    @property
    def _w(self):
        """host words [size, n2w] (downloaded from HBM on first use)"""
        h = self._st.host()
        return h if self._whole() else h[self._lo:self._lo + self.size]

    def _dw(self, dev):
        """device words [size, n2w] on `dev`: a view of the resident copy, the
        whole buffer uploaded once (then kept), or a temporary upload of a
        slice of a host-only buffer"""
        if self._whole() or self._st.on_device(dev):
            d = self._st.device(dev)
            return d if self._whole() else d[self._lo:self._lo + self.size]
        return resident.upload(self._w, dev)

    def _resident_on(self, dev):
        return dev is not None and self._st.on_device(dev)

    def to_device(self, device=None):
        """Keep a copy of the words in HBM of `device` (default: the
        context's own GPU), so following batched operations run there and
        leave their results there; returns self. No-op in host-buffer mode."""
        dev = resident.device_for(self.context) if device is None else device
        if dev is not None and self.size:
            self._st.device(dev)  # the whole storage: views keep sharing it
        return self

    @property
    def is_resident(self):
        """whether the words are held in HBM"""
        return self._st.d is not None

    @property
    def words(self):
        """uint32 [size, n2w] residues mod n^2 (C order over shape), read-only
        (write through arr[i] = ciphertext: the words may also live in HBM)"""
        v = self._w.view()
        v.flags.writeable = False
        return v

    @property
    def exponents(self):
        """int32 [size] exponents"""
        return self._e

    # ------------------------------------------------------------ ndarray-like surface
    @property
    def shape(self):
        return self._shape

    @property
    def ndim(self):
        return len(self._shape)

    @property
    def size(self):
        return self._e.shape[0]

    @property
    def dtype(self):
        """PaillierDtype (kind 'O'); np.asarray(arr).dtype is object, as for
        the reference's arrays"""
        return PaillierDtype() if _EADtypeBase is not object else np.dtype(object)

    @property
    def nbytes(self):
        return self.size * (self._st.n2w * 4 + 4)

    @property
    def T(self):
        return self.transpose()

    def __len__(self):
        if not self._shape:
            raise TypeError("len() of unsized object")
        return self._shape[0]

    def __repr__(self):
        return f"PaillierArray(shape={self._shape}, key_bits={None if self.context is None else self.context.n.bit_length()})"

    def _elem(self, i, raw=None):
        CT = _ct_type()
        e = int(self._e[i])
        if e == NA_EXP:
            return np.nan
        if raw is None:
            raw = int.from_bytes(self._w[i].tobytes(), "little")
        return CT(self.context, raw, e)

    def _take(self, flat_idx, shape):
        flat_idx = np.asarray(flat_idx, dtype=np.int64).reshape(-1)
        if self._st.d is not None:  # stays in HBM
            d = self._st.d if self._whole() else self._st.d[self._lo:self._lo + self.size]
            return PaillierArray.from_device(self.context, resident.take(d, flat_idx), self._e[flat_idx], shape)
        return PaillierArray.from_buffers(self.context, self._w[flat_idx], self._e[flat_idx], shape)

    def _index_map(self):
        return np.arange(self.size, dtype=np.int64).reshape(self._shape)

    def __getitem__(self, key):
        if self.ndim == 1:
            if isinstance(key, (int, np.integer)):
                i = int(key)
                if i < -self.size or i >= self.size:
                    raise IndexError(f"index {i} is out of bounds for axis 0 with size {self.size}")
                return self._elem(i % self.size)
            if isinstance(key, slice) and (key.step is None or key.step == 1):
                lo, hi, _ = key.indices(self.size)
                hi = max(lo, hi)
                return self._view(lo, self._e[lo:hi], (hi - lo,))
        if isinstance(key, tuple) and len(key) == self.ndim and all(isinstance(k, (int, np.integer)) for k in key):
            idx = np.ravel_multi_index(tuple(int(k) % s for k, s in zip(key, self._shape)), self._shape)
            return self._elem(int(idx))
        sel = self._index_map()[key]
        if np.ndim(sel) == 0:
            return self._elem(int(sel))
        return self._take(sel, sel.shape)

    def __setitem__(self, key, value):
        key = _unbox_key(key)
        sel = np.asarray(self._index_map()[key], dtype=np.int64)
        if _is_na(value):  # pandas' missing value (setitem / where / reindex)
            self._e[sel.reshape(-1)] = NA_EXP
            return
        src = _as_cipher(value)
        if src is None and isinstance(value, numbers.Number) and not isinstance(value, complex):
            # a plain number stored into a ciphertext column (pandas fillna(0),
            # core/tree/...: merge(...).fillna(0)): its unobfuscated encryption,
            # which adds exactly as the reference's number cell does
            # (paillier.py:93-102)
            src = _plain_cipher(self.context, value)
        if src is None:
            raise TypeError(f"can only assign PaillierCiphertext values, got {type(value)}")
        if not _same_key(src.context, self.context):
            raise ValueError("Adding two ciphertext with different keys.")
        src = src._aligned_words(self._st.n2w)
        ib = np.broadcast_to(src._index_map(), sel.shape).reshape(-1)
        self._st.host()[self._lo + sel.reshape(-1)] = src._w[ib]
        self._st.host_written()
        self._e[sel.reshape(-1)] = src._e[ib]

    def __iter__(self):
        if self.ndim == 0:
            raise TypeError("iteration over a 0-d array")
        if self.ndim == 1:
            raws = nat.words_to_ints(self._w) if self.size else []
            for i, r in enumerate(raws):
                yield self._elem(i, r)
        else:
            for i in range(self._shape[0]):
                yield self[i]

    def reshape(self, *shape, order="C"):
        if order not in ("C", "A"):
            raise _unsupported("reshape(order='F')")
        if len(shape) == 1 and isinstance(shape[0], (tuple, list)):
            shape = tuple(shape[0])
        new = np.empty(self._shape, dtype=np.bool_).reshape(shape).shape  # numpy's -1 / size rules
        return self._view(0, self._e, new)

    def flatten(self, order="C"):
        return self.reshape(-1).copy() if order in ("C", "A") else self.transpose().reshape(-1)

    def ravel(self, order="C"):
        return self.reshape(-1) if order in ("C", "A") else self.transpose().reshape(-1)

    def transpose(self, *axes):
        if self.ndim < 2:
            return self
        perm = self._index_map().transpose(*axes) if axes else self._index_map().T
        return self._take(perm, perm.shape)

    def squeeze(self, axis=None):
        return self.reshape(np.empty(self._shape, dtype=np.bool_).squeeze(axis).shape)

    def copy(self, order="C"):
        if self._st.d is not None:
            d = self._st.d if self._whole() else self._st.d[self._lo:self._lo + self.size]
            return PaillierArray.from_device(self.context, resident.clone(d), self._e.copy(), self._shape)
        return PaillierArray.from_buffers(self.context, self._w.copy(), self._e.copy(), self._shape)

    def _obfuscate_in_place(self):
        """Paillier.obfuscate on the array (paillier.py:419-431): every
        element re-randomised in place, views included"""
        ctx = self.context
        n2w = ops.n2w_of(ctx)
        if self._st.n2w != n2w:
            raise ValueError(f"ciphertext rows of {self._st.n2w} words, the key's n^2 has {n2w}")
        dev = resident.device_for(ctx)
        if self._resident_on(dev):
            new = resident.obfuscate(ctx.device_key(dev), self._dw(dev))
            if self._whole():
                self._st.d = new
            else:
                resident.put_rows(self._st.d, np.arange(self._lo, self._lo + self.size), new)
            self._st.h = None  # the host copy is stale
            return
        h = self._st.host()
        h[self._lo:self._lo + self.size] = ops.obfuscate_words(ctx, h[self._lo:self._lo + self.size])
        self._st.host_written()

    def tolist(self):
        return self._objects().tolist()

    def astype(self, dtype, copy=True):
        """astype(object): the reference's np.ndarray[object] of
        PaillierCiphertext (as np.asarray); other dtypes convert from it."""
        if isinstance(dtype, PaillierDtype) or dtype == PaillierDtype.name:
            return self.copy() if copy else self
        if np.dtype(dtype) == np.dtype(object):
            return self._objects()
        return self._objects().astype(dtype)

    def _objects(self):
        """The reference's representation: np.ndarray[object] of PaillierCiphertext."""
        out = np.empty(self.size, dtype=object)
        if self.size:
            for i, r in enumerate(nat.words_to_ints(self._w)):
                out[i] = self._elem(i, r)
        return out.reshape(self._shape)

    def __array__(self, dtype=None, copy=None):
        arr = self._objects()
        return arr if dtype is None or np.dtype(dtype) == np.dtype(object) else arr.astype(dtype)

    def __reduce__(self):
        return (PaillierArray.from_buffers, (self.context, self._w, self._e, self._shape))

    # ------------------------------------------------------------ pandas ExtensionArray
    # (pandas/core/arrays/base.py's interface; 1-D arrays, as pandas uses them)
    @classmethod
    def _from_sequence(cls, scalars, *, dtype=None, copy=False):
        if isinstance(scalars, PaillierArray):
            return scalars.copy() if copy else scalars
        arr = np.empty(len(scalars), dtype=object)
        arr[:] = list(scalars)
        na = np.array([_is_na(v) for v in arr], dtype=bool)
        CT = _ct_type()
        if not all(isinstance(v, CT) for v in arr[~na]):
            raise TypeError("PaillierArray holds PaillierCiphertext elements")
        if not na.any():
            return cls(arr)
        if na.all():
            raise TypeError("PaillierArray._from_sequence: no ciphertext to take the key from")
        first = arr[~na][0]
        arr[na] = first  # placeholders, then marked missing
        out = cls(arr)
        out._e[na] = NA_EXP
        return out

    @classmethod
    def _from_factorized(cls, values, original):
        raise NotImplementedError("factorizing ciphertexts is not supported")

    @classmethod
    def _concat_same_type(cls, to_concat):
        parts = [p.reshape(-1) for p in to_concat]
        ctxs = [p.context for p in parts if p.context is not None]
        if not ctxs:
            n2w = max(p._st.n2w for p in parts)
            parts = [p._aligned_words(n2w) for p in parts]
            return cls.from_buffers(None, np.concatenate([p._w for p in parts]),
                                    np.concatenate([p._e for p in parts]))
        ctx = _ctx_of(*parts)
        n2w = ops.n2w_of(ctx)
        parts = [p._aligned_words(n2w) for p in parts]
        e = np.concatenate([p._e for p in parts])
        dev = _res_dev(ctx, *parts)
        if dev is not None:
            return cls.from_device(ctx, resident.cat([p._dw(dev) for p in parts]), e)
        return cls.from_buffers(ctx, np.concatenate([p._w for p in parts]), e)

    def isna(self):
        return (self._e == NA_EXP).reshape(self._shape)

    def _has_na(self):
        return self.size > 0 and int(self._e.min()) == NA_EXP

    def take(self, indices, allow_fill=False, fill_value=None):
        """pandas take: -1 gives a missing entry when allow_fill (an outer
        merge's reindex), numpy's negative indexing otherwise"""
        idx = np.asarray(indices, dtype=np.int64).reshape(-1)
        n = self.size
        if allow_fill:
            if idx.size and idx.min() < -1:
                raise ValueError("take: indices below -1 with allow_fill")
            fill = idx == -1
        else:
            idx = np.where(idx < 0, idx + n, idx)
            fill = None
        if idx.size and idx.max() >= n:
            raise IndexError(f"take: index {int(idx.max())} out of bounds for size {n}")
        if fill is None or not fill.any():
            return self._take(idx, (idx.size,))
        if n == 0:  # every entry missing
            out = PaillierArray.from_buffers(self.context, np.zeros((idx.size, self._st.n2w), np.uint32),
                                             np.full(idx.size, NA_EXP, np.int32))
        else:
            out = self._take(np.where(fill, 0, idx), (idx.size,))
        if fill_value is None or _is_na(fill_value):
            out._e[fill] = NA_EXP
        else:
            out[np.nonzero(fill)[0]] = fill_value
        return out

    def _values_for_argsort(self):
        raise TypeError("ciphertexts have no order")

    def __eq__(self, other):
        """element-wise: equal residues and exponents (the reference's object
        arrays compare element identity; pandas needs a value comparison)"""
        co = _as_cipher(other)
        if co is None:
            return np.zeros(self._shape, dtype=bool)
        ia, ib, shape = _bcast(self, co)
        wa, ea = _rows(self, ia)
        wb, eb = _rows(co._aligned_words(self._st.n2w), ib)
        return (np.all(wa == wb, axis=1) & (ea == eb) & (ea != NA_EXP)).reshape(shape)

    def __ne__(self, other):
        return ~self.__eq__(other)

    __hash__ = None

    def _reduce(self, name, *, skipna=True, keepdims=False, **kwargs):
        """Series.sum() over a ciphertext column = np.sum (order-free fold)"""
        if name != "sum":
            raise TypeError(f"cannot perform {name} with type {self.dtype}")
        x = self.reshape(-1)
        if x._has_na():
            if not skipna:
                return np.nan
            x = x[~x.isna()]
        if x.size == 0:
            return 0  # the reference's empty object sum
        s = _sum(x, None, False)
        if keepdims:
            return PaillierArray(np.array([s], dtype=object))
        return s

    def _groupby_op(self, *, how, has_dropped_na, min_count, ngroups, ids, **kwargs):
        """groupby(...).sum() of a ciphertext column: ONE segmented product
        (xhe_segprod) over the rows sorted stably by group, equal bit for bit
        to pandas' object group_sum (a left fold per group in row order,
        skipping NaN; groups with fewer than min_count values give NaN, empty
        groups the reference's int 0 as the encryption of 0). Other
        reductions: NotImplementedError, so pandas runs its per-group Python
        fallback over the ciphertext objects."""
        if how != "sum" or self.ndim != 1 or self.context is None:
            raise NotImplementedError(f"groupby {how} over ciphertexts")
        ctx = self.context
        ids = np.asarray(ids).reshape(-1)
        valid = ids >= 0
        if self._has_na():
            valid &= ~self.isna()
        key = np.where(valid, ids, ngroups)
        # stable sort by group: radix sort on narrow keys (numpy's stable sort of <= 16-bit ints)
        key = key.astype(np.uint16 if ngroups < (1 << 16) - 1 else np.int64)
        nvalid = int(np.count_nonzero(valid))
        order = np.argsort(key, kind="stable")[:nvalid]
        cnt = np.bincount(ids[valid], minlength=ngroups).astype(np.int64)
        seg = np.zeros(ngroups + 1, dtype=np.int64)
        np.cumsum(cnt, out=seg[1:])
        n2w = ops.n2w_of(ctx)
        x = self._aligned_words(n2w)
        dev = resident.device_for(ctx, -1, x._st.count, 4 * n2w)
        if dev is not None and (x._resident_on(dev) or x.size > SMALL):
            x.to_device(dev)  # the whole column's words, once (every later call reads them in HBM)
        if dev is not None and (x._resident_on(dev) or nvalid <= SMALL):
            dw, e = _drows(x, order, dev)
            rd, re = ops.segment_sums_dev(ctx, ctx.device_key(dev), dw, e, seg, fold=True)
            out = PaillierArray.from_device(ctx, rd, re, (ngroups,))
        else:
            w, e = _rows(x, order)
            rw, re = ops.segment_sums_words(ctx, w, e, seg, fold=True)
            out = _result(ctx, rw, re, (ngroups,))
        short = cnt < max(int(min_count), 1) if min_count > 0 else None
        if short is not None and short.any():
            out._e[short] = NA_EXP
        return out

    def _aligned_words(self, n2w):
        """self with n2w-word rows (arrays decoded without a context keep the
        wire's width)."""
        if self._st.n2w == n2w:
            return self
        if self._w.shape[1] > n2w:
            if self._w[:, n2w:].any():
                raise ValueError("ciphertext wider than the key's n^2")
            w = np.ascontiguousarray(self._w[:, :n2w])
        else:
            w = np.zeros((self.size, n2w), dtype=np.uint32)
            w[:, :self._w.shape[1]] = self._w
        return PaillierArray.from_buffers(self.context, w, self._e, self._shape)

    # ------------------------------------------------------------ reductions
    def sum(self, axis=None, dtype=None, out=None, keepdims=False, initial=None, where=None):
        if out is not None or dtype not in (None, object) or where is not None or initial is not None:
            return _obj_call(np.sum, (self,), dict(axis=axis, dtype=dtype, out=out, keepdims=keepdims,
                                                   initial=initial, where=where))
        return _sum(self, axis, keepdims)

    # ------------------------------------------------------------ operators
    def __add__(self, other):
        return _dispatch(_add, self, other, np.add)

    def __radd__(self, other):
        return _dispatch(_add, other, self, np.add)

    def __sub__(self, other):
        return _dispatch(_sub, self, other, np.subtract)

    def __rsub__(self, other):
        return _dispatch(_sub, other, self, np.subtract)

    def __mul__(self, other):
        return _dispatch(_mul, self, other, np.multiply)

    def __rmul__(self, other):
        return _dispatch(_mul, other, self, np.multiply)

    def __truediv__(self, other):
        return _dispatch(_div, self, other, np.true_divide)

    def __rtruediv__(self, other):
        return _dispatch(_div, other, self, np.true_divide)

    def __matmul__(self, other):
        return _dispatch(_matmul, self, other, np.matmul)

    def __rmatmul__(self, other):
        return _dispatch(_matmul, other, self, np.matmul)

    def __neg__(self):
        return _mul(self, -1)

    def __pos__(self):
        return self

    # ------------------------------------------------------------ numpy protocols
    def __array_ufunc__(self, ufunc, method, *inputs, out=None, **kwargs):
        if method == "__call__" and out is None and not kwargs:
            fn = _UFUNCS.get(ufunc)
            if fn is not None:
                try:
                    return fn(*inputs)
                except _Fallback:
                    pass
        if out is not None:
            kwargs["out"] = tuple(_plain(o) for o in out)
        return _wrap(getattr(ufunc, method)(*[_plain(x) for x in inputs], **kwargs))

    def __array_function__(self, func, types, args, kwargs):
        fn = _FUNCS.get(func)
        if fn is not None:
            try:
                return fn(*args, **kwargs)
            except _Fallback:
                pass
        return _obj_call(func, args, kwargs)


def _unsupported(what):
    return NotImplementedError(f"PaillierArray.{what} is not supported")


def _is_na(v):
    """pandas' missing-value scalars (None, NaN, pd.NA)"""
    if v is None:
        return True
    if isinstance(v, (float, np.floating)):
        return bool(np.isnan(v))
    if _EABase is not object:
        import pandas as pd
        return v is pd.NA or v is pd.NaT
    return False


def _unbox_key(key):
    """pandas array keys (BooleanArray / IntegerArray / Index) -> numpy"""
    if hasattr(key, "to_numpy") and not isinstance(key, (PaillierArray, np.ndarray)):
        return key.to_numpy()
    return key


def _plain_cipher(ctx, value):
    """the unobfuscated encryption of a number at its precision=None exponent,
    1 + n m mod n^2 (paillier.py:93-102, 283), as a 0-d PaillierArray - on the
    host (no device call for a fill value)"""
    if ctx is None:
        return None
    from .encoder import PaillierEncoder
    v = value.item() if isinstance(value, np.generic) else value
    v = int(v) if isinstance(v, bool) else v
    e = PaillierEncoder.cal_exponent(v, precision=None)
    m = int(PaillierEncoder.encode_single(ctx, v, e))
    ct = _ct_type()(ctx, (1 + ctx.n * m) % ctx.n_square, int(e))
    return PaillierArray(np.array(ct, dtype=object).reshape(()))


def _check_no_na(*xs):
    """arithmetic on a missing entry raises, as the reference's ciphertext +
    NaN does (encrypting NaN, paillier.py:93-98)"""
    for x in xs:
        if isinstance(x, PaillierArray) and x._has_na():
            raise ValueError("cannot convert float NaN to integer: missing ciphertext entries (fillna first)")


def _n2w(ctx, raws=()):
    if ctx is not None:
        return ops.n2w_of(ctx)
    bits = max((int(r).bit_length() for r in raws), default=1)
    for k in (2048, 3072, 4096, 8192):
        if bits <= 2 * k:
            return 2 * k // 32
    return (bits + 31) // 32


def _plain(x):
    """PaillierArray -> the reference's object array (recursively in lists)."""
    if isinstance(x, PaillierArray):
        return x._objects()
    if isinstance(x, (list, tuple)):
        return type(x)(_plain(v) for v in x)
    return x


def _obj_call(func, args, kwargs):
    return _wrap(func(*[_plain(a) for a in args], **{k: _plain(v) for k, v in kwargs.items()}))


def _wrap(res):
    """Object arrays of ciphertexts of one key come back as PaillierArray;
    anything else is returned as numpy made it."""
    if isinstance(res, np.ndarray) and res.dtype == object and res.size:
        CT = _ct_type()
        flat = res.reshape(-1)
        if all(isinstance(c, CT) for c in flat):
            ctx = flat[0].context
            if all(_same_key(c.context, ctx) for c in flat):
                return PaillierArray(res)
    return res


def _as_cipher(x):
    """x as a PaillierArray when it is ciphertext-only, else None."""
    if isinstance(x, PaillierArray):
        return x
    CT = _ct_type()
    if isinstance(x, CT):
        return PaillierArray(np.array(x, dtype=object).reshape(()))
    if isinstance(x, (list, tuple)) or (isinstance(x, np.ndarray) and x.dtype == object):
        arr = np.asarray(x, dtype=object) if not (isinstance(x, np.ndarray)) else x
        if arr.size and all(isinstance(c, CT) for c in arr.reshape(-1)):
            return PaillierArray(arr)
    return None


def _as_plain(x):
    """x as a numeric array of plaintext scalars, or None. Python numbers and
    numeric ndarrays (numpy casts their elements to Python scalars in the
    reference's object loops, so float32 elements are exact floats there)."""
    if isinstance(x, PaillierArray) or isinstance(x, _ct_type()):
        return None
    if isinstance(x, bool) or isinstance(x, (int, float)) and not isinstance(x, np.generic):
        return np.asarray(x, dtype=object if isinstance(x, int) and abs(x) >= 2 ** 63 else None)
    if isinstance(x, np.generic) and x.dtype.kind in "biuf":
        return np.asarray(x)
    if isinstance(x, np.ndarray):
        if x.dtype.kind in "biuf":
            return x
        if x.dtype == object and x.size and all(isinstance(v, (int, float)) for v in x.reshape(-1)):
            return x
    if isinstance(x, (list, tuple)):
        try:
            a = np.asarray(x)
        except (ValueError, TypeError):
            return None
        return _as_plain(a) if a.dtype.kind in "biuf" or a.dtype == object else None
    return None


def _dispatch(fn, a, b, ufunc):
    try:
        return fn(a, b)
    except _Fallback:
        return _wrap(ufunc(_plain(a), _plain(b)))


def _bcast(a, b):
    """broadcast flat index maps of two operands -> (ia, ib, shape); an
    operand whose shape is the result's gets None (the identity map)"""
    sa = a.shape if hasattr(a, "shape") else ()
    sb = b.shape if hasattr(b, "shape") else ()
    shape = np.broadcast_shapes(sa, sb)

    def imap(s):
        if tuple(s) == tuple(shape):
            return None
        return np.broadcast_to(np.arange(int(np.prod(s, dtype=np.int64)), dtype=np.int64).reshape(s), shape).reshape(-1)
    return imap(sa), imap(sb), shape


def _identity(idx, size):
    return idx is None or (idx.shape[0] == size and (size == 0 or (idx[0] == 0 and np.all(np.diff(idx) == 1))))


def _at(flat, idx):
    return flat if idx is None else flat[idx]


def _rows(x, idx):
    """rows of x at idx, without a copy when idx is the identity"""
    if _identity(idx, x.size):
        return x._w, x._e
    return x._w[idx], x._e[idx]


def _drows(x, idx, dev):
    """_rows on device words (resident.py)"""
    d = x._dw(dev)
    if _identity(idx, x.size):
        return d, x._e
    return resident.take(d, idx), x._e[idx]


SMALL = 1 << 16  # host-only operands up to this many elements are uploaded (no host pipeline set-up)


def _res_dev(ctx, *xs):
    """The GPU to run a batched op on in HBM: the context's own GPU when some
    ciphertext operand is resident there, or when the host-only operands are
    small (uploading them costs less than the host pipeline's set-up); results
    then stay in HBM. None -> the host-buffer path (xfl_amd.paillier.ops),
    which overlaps the copies of large host arrays with the kernels."""
    dev = resident.device_for(ctx)
    if dev is None:
        return None
    xs = [x for x in xs if x is not None]
    if any(x._resident_on(dev) for x in xs) or sum(x.size for x in xs) <= SMALL:
        return dev
    return None


def _ctx_of(*xs):
    ctx = None
    for x in xs:
        if x.context is not None:
            if ctx is not None and not _same_key(ctx, x.context):
                raise ValueError("Adding two ciphertext with different keys.")
            ctx = ctx or x.context
    if ctx is None:
        raise ValueError("ciphertext array without a context: pass one to Paillier.ciphertext_from")
    return ctx


def _result(ctx, w, e, shape):
    return PaillierArray.from_buffers(ctx, w, e, shape)


# ------------------------------------------------------------ element-wise ops
def _encrypt_plain(ctx, vals):
    """Paillier.encrypt(scalar, precision=None, obfuscation=False) of every
    element (the scalar operand of PaillierCiphertext.__add__, paillier.py:96-98)."""
    from .paillier import Paillier
    arr = Paillier.encrypt(ctx, np.asarray(vals).reshape(-1) if np.ndim(vals) else np.asarray(vals).reshape(1),
                           precision=None, max_exponent=None, obfuscation=False)
    return arr


def _add(a, b):
    """a + b with the reference's semantics (paillier.py:88-126)."""
    ca, cb = _as_cipher(a), _as_cipher(b)
    _check_no_na(ca, cb)
    if ca is not None and cb is not None:
        ctx = _ctx_of(ca, cb)
        n2w = ops.n2w_of(ctx)
        ca, cb = ca._aligned_words(n2w), cb._aligned_words(n2w)
        ia, ib, shape = _bcast(ca, cb)
        return _add_rows(ctx, ca, ia, cb, ib, shape)
    if ca is None and cb is not None:
        a, b, ca, cb = b, a, cb, ca
    if ca is None:
        raise _Fallback()
    p = _as_plain(b)
    if p is None:
        if isinstance(b, (str, bytes)) or not hasattr(b, "__len__"):
            raise TypeError(f"Adding data of type {type(b)} not supported.")
        raise _Fallback()
    ctx = _ctx_of(ca)
    ca = ca._aligned_words(ops.n2w_of(ctx))
    ia, ib, shape = _bcast(ca, p)
    nout = int(np.prod(shape, dtype=np.int64))
    P = _at(np.asarray(p).reshape(-1), ib) if p.ndim else np.repeat(np.asarray(p).reshape(1), nout)
    enc = _plain_aligned(ctx, ca, ia, P)
    if enc is None:
        enc = _encrypt_plain(ctx, P)
    return _add_rows(ctx, ca, ia, enc, None, shape)


def _plain_aligned(ctx, ca, ia, P):
    """The scalar operand of ciphertext + scalar, encrypted and already at the
    sum's exponent. The reference encrypts the scalar unobfuscated, c = 1 + n m
    (paillier.py:95-101, 266-268), and where its exponent is the larger one
    _decrease_exponent_to raises c to 2^d (paillier.py:79-86, 106-119). Since
    (1 + n m)^(2^d) = 1 + n (m 2^d mod n) mod n^2 (the negative branch's
    c^(2^d - n) as well), that is the plain encryption of m 2^d, the scalar
    encoded at the ciphertext's exponent: a word shift on the host instead of
    d squarings mod n^2 on the device. Device path only; None (encrypt, then
    align, as before) off it, for scalars outside the vectorised encoder's
    domain, or when m 2^d would come near n."""
    dev = _res_dev(ctx, ca)
    if dev is None:
        return None
    ec = ca._e.astype(np.int64)[ia] if ia is not None else ca._e.astype(np.int64).reshape(-1)
    enc = _encode_at(ctx, P, ec)
    if enc is None:
        return None
    m, enew = enc
    k, nw = m.shape
    if k <= 64:
        # 1 + n m (< n^2, paillier.py:266-268) on the host (~5 us an element,
        # overlapping the device's queue): for the LR step's 15 elements
        # cheaper than the one-lane k_raw_enc launch behind it (~85 us)
        n = ctx.n
        ct = resident.upload(nat.ints_to_words([1 + n * v for v in nat.words_to_ints(m)], 2 * nw), dev)
    else:
        ct = resident.encrypt_encoded(ctx.device_key(dev), m, False)
    return PaillierArray.from_device(ctx, ct, enew.astype(np.int32), (k,))


def _encode_at(ctx, P, ec):
    """encode_single of every scalar of P at exponent min(its own, ec)
    (encoder.py:48-54 at the aligned exponent, < n/8): (m words [k, nw],
    exponents), or None outside the vectorised encoder's domain or when a
    value would come near n"""
    if P.dtype == object:
        return None
    vec = _encode_scalars_vec(P)
    if vec is None:
        return None
    kabs, neg, ep = (v.reshape(-1) for v in vec)
    if kabs.size == 0:
        return None
    ec = np.broadcast_to(np.asarray(ec, dtype=np.int64).reshape(-1), kabs.shape)
    enew = np.minimum(ep, ec)
    words, kbits = _shifted_words(kabs, ep - enew)
    if kbits > ctx.n.bit_length() - 3:
        return None
    nw = ops.nw_of(ctx)
    m = np.zeros((kabs.size, nw), np.uint32)
    m[:, :words.shape[1]] = words
    if neg.any():
        m[neg] = _n_minus(ctx, m[neg], nw)
    return m, enew


def _n_minus(ctx, x, nw):
    """n - x for host words x [k, nw] (every x < n): Python ints for small
    batches, else a borrow chain vectorised over the rows"""
    if x.shape[0] <= 256:
        n = ctx.n
        return nat.ints_to_words([n - v for v in nat.words_to_ints(x)], nw)
    nwd = nat.ints_to_words([ctx.n], nw)[0].astype(np.int64)
    out = np.empty_like(x)
    br = np.zeros(x.shape[0], np.int64)
    for j in range(nw):
        v = nwd[j] - x[:, j].astype(np.int64) - br
        br = (v < 0).astype(np.int64)
        out[:, j] = (v + (br << 32)).astype(np.uint32)
    return out


def _add_rows(ctx, ca, ia, cb, ib, shape):
    """ca[ia] + cb[ib] element-wise (paillier.py:106-123): in HBM when an
    operand is resident there, else through host buffers"""
    dev = _res_dev(ctx, ca, cb)
    if dev is None:
        wa, ea = _rows(ca, ia)
        wb, eb = _rows(cb, ib)
        w, e = ops.add_words(ctx, wa, ea, wb, eb)
        return _result(ctx, w, e, shape)
    da, ea = _drows(ca, ia, dev)
    db, eb = _drows(cb, ib, dev)
    n = ea.shape[0]
    if n == 0:
        return _result(ctx, np.zeros((0, ops.n2w_of(ctx)), np.uint32), np.zeros(0, np.int32), shape)
    lo, hi = min(int(ea.min()), int(eb.min())), max(int(ea.max()), int(eb.max()))
    dk = ctx.device_key(dev)
    if lo == hi:  # one exponent throughout (the usual case): no alignment, nothing to upload
        return PaillierArray.from_device(ctx, resident.mulmod(dk, da, None, db, None, 0), np.full(n, lo, np.int32),
                                         shape)
    wide = np.int32 if hi - lo < (1 << 31) else np.int64
    dmax = int(np.max(np.abs(ea.astype(wide) - eb.astype(wide))))
    out = resident.mulmod(dk, da, ea, db, eb, dmax)
    return PaillierArray.from_device(ctx, out, np.minimum(ea, eb), shape)


def _neg_plain(p):
    """other * (-1) of a plaintext operand (paillier.py:128-132), elementwise"""
    if p.dtype == object:
        return np.vectorize(lambda v: v * (-1), otypes=[object])(p)
    if p.dtype.kind == "u" or p.dtype == np.bool_:
        return (-p.astype(object)) if p.dtype.kind == "u" else -(p.astype(np.int64))
    return -p


def _sub(a, b):
    """a - b = a + b * (-1); scalar - ct = (-1) * ct + scalar (paillier.py:128-132)."""
    cb = _as_cipher(b)
    if cb is not None:
        return _add(a, _mul(cb, -1))
    if _as_cipher(a) is None:
        raise _Fallback()
    p = _as_plain(b)
    if p is None:
        raise _Fallback()
    return _add(a, _neg_plain(p))


def _encode_scalars_vec(X):
    """Vectorised PaillierEncoder.cal_exponent(precision=None) + encode_single
    (encoder.py:29-54) of a plain numeric array, as (|k|, k negative, e):
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
    if X.dtype.kind in "iub" and X.dtype.itemsize <= 8:
        if X.dtype.kind == "u" and X.size and int(X.max()) >= 2 ** 63:
            return None
        x = X.astype(np.int64)
        if X.dtype.kind == "i" and np.any(x == np.iinfo(np.int64).min):
            return None
        return np.abs(x), x < 0, np.zeros(X.shape, dtype=np.int64)
    return None


def _encode_scalars(ctx, P):
    """(|k| words, negative flags, exponents) of every scalar of P (flat)."""
    from .encoder import PaillierEncoder
    vec = _encode_scalars_vec(P) if P.dtype != object else None
    if vec is not None:
        kabs, neg, e = vec
        return kabs.reshape(-1), neg.reshape(-1), e.reshape(-1)
    thr = ctx.min_value_for_negative
    ks, neg, es = [], [], []
    for s in P.reshape(-1):
        s = s.item() if isinstance(s, np.generic) else s
        e = PaillierEncoder.cal_exponent(s, precision=None)
        k = int(PaillierEncoder.encode_single(ctx, s, e))
        if k >= thr:
            ks.append(ctx.n - k)
            neg.append(True)
        else:
            ks.append(k)
            neg.append(False)
        es.append(int(e))
    kbits = max(1, max(k.bit_length() for k in ks))
    return nat.ints_to_words(ks, (kbits + 31) // 32), np.array(neg, dtype=bool), np.array(es, dtype=np.int64)


def _mul(a, b):
    """ciphertext * scalar element-wise (paillier.py:134-187)."""
    ca, cb = _as_cipher(a), _as_cipher(b)
    if ca is not None and cb is not None:
        raise TypeError("Cannot multiply one ciphertext with another ciphertext, try multiply a scalar.")
    if ca is None and cb is not None:
        a, b, ca = b, a, cb
    if ca is None:
        raise _Fallback()
    _check_no_na(ca)
    p = _as_plain(b)
    if p is None:
        if isinstance(b, (str, bytes)) or not hasattr(b, "__len__"):
            raise TypeError(f"Precision type {type(None)} not supported.")
        raise _Fallback()
    ctx = _ctx_of(ca)
    ca = ca._aligned_words(ops.n2w_of(ctx))
    ia, ib, shape = _bcast(ca, p)
    nout = int(np.prod(shape, dtype=np.int64))
    P = _at(np.asarray(p).reshape(-1), ib) if np.ndim(p) else np.repeat(np.asarray(p).reshape(1), nout)
    kabs, neg, ek = _encode_scalars(ctx, P)
    dev = _res_dev(ctx, ca)
    if dev is not None:
        da, ea = _drows(ca, ia, dev)
        e = (ea.astype(np.int64) + ek).astype(np.int32)
        if e.shape[0] == 0:
            return _result(ctx, np.zeros((0, ops.n2w_of(ctx)), np.uint32), e, shape)
        return PaillierArray.from_device(ctx, ops.raw_mul_dev(ctx.device_key(dev), da, kabs, neg), e, shape)
    wa, ea = _rows(ca, ia)
    w = ops.raw_mul_words(ctx, wa, kabs, neg)
    e = (ea.astype(np.int64) + ek).astype(np.int32)
    return _result(ctx, w, e, shape)


def _div(a, b):
    """ct / s = ct * (1 / s) (paillier.py:150-151), 1/s in float64 per element."""
    if _as_cipher(b) is not None or _as_cipher(a) is None:
        raise _Fallback()
    p = _as_plain(b)
    if p is None:
        raise _Fallback()
    if p.dtype == object:
        inv = np.vectorize(lambda s: 1 / s, otypes=[object])(p)
    else:
        inv = 1.0 / np.asarray(p, dtype=np.float64)
    return _mul(a, inv)


# ------------------------------------------------------------ reductions
def _sum(x, axis=None, keepdims=False):
    """np.sum over ciphertexts: per output element the order-free product
    prod c_i^(2^(e_i - e_min)) (paillier.py:79-123 folded)."""
    ctx = _ctx_of(x)
    _check_no_na(x)
    x = x._aligned_words(ops.n2w_of(ctx))
    if x.ndim == 0:
        return x._elem(0)
    if axis is None:
        axes = tuple(range(x.ndim))
    else:
        axes = tuple(sorted(a % x.ndim for a in (axis if isinstance(axis, tuple) else (axis,))))
    keep = [d for d in range(x.ndim) if d not in axes]
    perm = x._index_map().transpose(keep + list(axes))
    out_shape = tuple(x.shape[d] for d in keep)
    nseg = int(np.prod(out_shape, dtype=np.int64))
    seglen = x.size // nseg if nseg else 0
    if seglen == 0:
        raise _Fallback()  # empty reduction: the reference's object sum gives int 0
    order = None if keep + list(axes) == list(range(x.ndim)) else perm.reshape(-1)
    seg = np.arange(nseg + 1, dtype=np.int64) * seglen
    dev = _res_dev(ctx, x)
    # numpy's add.reduce over an object array is a left fold in this order
    if dev is not None:
        dw, e = _drows(x, order, dev)
        rd, re = ops.segment_sums_dev(ctx, ctx.device_key(dev), dw, e, seg, fold=True)
        res = lambda shp: PaillierArray.from_device(ctx, rd, re, shp)  # noqa: E731
    else:
        w, e = _rows(x, order)
        rw, re = ops.segment_sums_words(ctx, w, e, seg, fold=True)
        res = lambda shp: _result(ctx, rw, re, shp)  # noqa: E731
    if keepdims:
        out_shape = tuple(1 if d in axes else x.shape[d] for d in range(x.ndim))
    if not out_shape:
        return res((1,))._elem(0)
    return res(out_shape)


def _f_sum(a, axis=None, dtype=None, out=None, keepdims=False, initial=None, where=None):
    c = _as_cipher(a)
    if c is None or out is not None or dtype not in (None, object) or initial is not None or where is not None:
        raise _Fallback()
    return _sum(c, axis, keepdims)


def _f_concatenate(arrays, axis=0, out=None, dtype=None, casting="same_kind"):
    if out is not None or dtype not in (None, object):
        raise _Fallback()
    cs = [_as_cipher(a) for a in arrays]
    if not cs or any(c is None for c in cs):
        raise _Fallback()
    ctx = _ctx_of(*cs)
    n2w = ops.n2w_of(ctx)
    cs = [c._aligned_words(n2w) for c in cs]
    if axis is None:
        cs = [c.reshape(-1) for c in cs]
        axis = 0
    idx_parts, off = [], 0
    for c in cs:
        idx_parts.append(c._index_map() + off)
        off += c.size
    idx = np.concatenate(idx_parts, axis=axis)
    e = np.concatenate([c._e for c in cs])
    flat = idx.reshape(-1)
    dev = _res_dev(ctx, *cs)
    if dev is not None:
        d = resident.cat([c._dw(dev) for c in cs])
        return PaillierArray.from_device(ctx, d if _identity(flat, d.shape[0]) else resident.take(d, flat), e[flat],
                                         idx.shape)
    w = np.concatenate([c._w for c in cs]) if cs else np.zeros((0, n2w), np.uint32)
    return _result(ctx, w[flat], e[flat], idx.shape)


def _f_stack(arrays, axis=0, out=None, dtype=None, casting="same_kind"):
    if out is not None or dtype not in (None, object) or axis != 0:
        raise _Fallback()
    cs = [_as_cipher(a) for a in arrays]
    if not cs or any(c is None for c in cs) or len({c.shape for c in cs}) != 1:
        raise _Fallback()
    return _f_concatenate([c.reshape((1,) + c.shape) for c in cs], axis=0)


def _f_reshape(a, *args, **kw):
    if isinstance(a, PaillierArray):
        newshape = kw.pop("newshape", kw.pop("shape", args[0] if args else None))
        return a.reshape(newshape, order=kw.get("order", "C"))
    raise _Fallback()


def _f_ravel(a, order="C"):
    if isinstance(a, PaillierArray):
        return a.ravel(order)
    raise _Fallback()


def _f_shape(a):
    return a.shape


def _f_ndim(a):
    return a.ndim


def _f_size(a, axis=None):
    return a.size if axis is None else a.shape[axis]


def _f_copy(a, order="K", subok=False):
    return a.copy()


def _f_transpose(a, axes=None):
    return a.transpose(*(axes or ()))


# ------------------------------------------------------------ matmul
def _matmul(a, b):
    """enc[B] @ X[B, D] (logistic_regression/trainer.py:166) and X[D, B] @
    enc[B]: per output j the multi-exponentiation prod_i base_i^(k'_ij *
    2^(d_ij)) with base_i = c_i or c_i^-1 (negative scalars) and d_ij aligning
    e_i + e_kij to the column minimum = the reference's object-dtype dot
    product (a fold of __mul__ + __add__) bit for bit."""
    ca, cb = _as_cipher(a), _as_cipher(b)
    if ca is not None and cb is not None:
        raise TypeError("Cannot multiply one ciphertext with another ciphertext, try multiply a scalar.")
    if ca is not None:
        X = _as_plain(b)
        if X is None or ca.ndim != 1 or np.ndim(X) != 2 or X.shape[0] != ca.shape[0] or ca.size == 0:
            raise _Fallback()
        return _matvec(ca, X)
    if cb is not None:
        X = _as_plain(a)
        if X is None or cb.ndim != 1 or np.ndim(X) != 2 or X.shape[1] != cb.shape[0] or cb.size == 0:
            raise _Fallback()
        return _matvec(cb, np.asarray(X).T)
    raise _Fallback()


def _matvec(A, X):
    ctx = _ctx_of(A)
    _check_no_na(A)
    A = A._aligned_words(ops.n2w_of(ctx))
    Bn, D = X.shape
    cexp = A._e.astype(np.int64)
    kw_, neg, e_k = _encode_scalars(ctx, np.asarray(X))
    kvec = kw_.ndim == 1  # int64 |k| from the vectorised encoder
    ks = None if kvec else nat.words_to_ints(kw_)  # |k_ij|, row-major [B, D]
    neg = neg.reshape(Bn, D)
    ex = cexp[:, None] + e_k.reshape(Bn, D)
    emin = ex.min(axis=0)
    need_inv = np.nonzero(neg.any(axis=1))[0]
    dev = _res_dev(ctx, A)
    inv_slot = np.full(Bn, -1, dtype=np.int64)
    if dev is not None:
        dk = ctx.device_key(dev)
        bases = A._dw(dev)
        if need_inv.size:
            inv = resident.invert(dk, resident.take(bases, need_inv))
            inv_slot[need_inv] = Bn + np.arange(need_inv.size)
            bases = resident.cat([bases, inv])
    else:
        bases = A._w
        if need_inv.size:
            one = np.zeros((need_inv.size, 1), dtype=np.uint32)
            one[:, 0] = 1
            inv = ops.powmod_words(ctx, A._w[need_inv], one, 1, invert_first=True)
            inv_slot[need_inv] = Bn + np.arange(need_inv.size)
            bases = np.concatenate([A._w, inv])
    rows = np.arange(Bn, dtype=np.int64)
    idx = np.where(neg, inv_slot[:, None], rows[:, None]).T.astype(np.int32)  # [D, B]
    shift = (ex - emin[None, :]).T  # [D, B]
    if kvec:
        kwords, kbits = _shifted_words(np.ascontiguousarray(kw_.reshape(Bn, D).T), shift)
    else:
        exps = [ks[i * D + j] << int(shift[j, i]) for j in range(D) for i in range(Bn)]
        kbits = max(1, max(k.bit_length() for k in exps))
        kwords = nat.ints_to_words(exps, (kbits + 31) // 32)
    if dev is not None:
        r = resident.multiexp(dk, bases, idx, kwords, kbits)
        return PaillierArray.from_device(ctx, r, emin.astype(np.int32), (D,))
    r = ops.multiexp_words(ctx, bases, idx, kwords, kbits)
    return _result(ctx, r, emin.astype(np.int32), (D,))


def _shifted_words(k, shift):
    """words of k << shift for int64 k >= 0 (< 2^63) and shifts >= 0, same
    shape -> (uint32 [k.size, kw], kbits) with every value < 2^kbits: the
    aligned multi-exponentiation exponents without a Python int per term"""
    k = k.reshape(-1).astype(np.uint64)
    s = shift.reshape(-1).astype(np.int64)
    nz = k != 0
    if not nz.any():
        return np.zeros((k.size, 1), np.uint32), 1
    kb = np.frexp(k[nz].astype(np.float64))[1].astype(np.int64)  # >= the bit length (float rounding up)
    kbits = int((kb + s[nz]).max())
    kw = (kbits + 31) // 32
    out = np.zeros((k.size, kw + 3), np.uint32)
    w0 = np.where(nz, s // 32, 0)  # zero terms may carry any shift
    b = (s % 32).astype(np.uint64)
    lo = k << b  # < 2^94 in all: three words from word w0 (numpy's uint64 shift wraps)
    hi = np.where(b > 0, k >> (np.uint64(64) - np.where(b > 0, b, np.uint64(1))), np.uint64(0))
    r = np.arange(k.size)
    out[r, w0] = (lo & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    out[r, w0 + 1] = (lo >> np.uint64(32)).astype(np.uint32)
    out[r, w0 + 2] = hi.astype(np.uint32)
    return np.ascontiguousarray(out[:, :kw]), kbits


_UFUNCS = {np.add: _add, np.subtract: _sub, np.multiply: _mul, np.true_divide: _div, np.matmul: _matmul,
           np.negative: lambda a: _mul(a, -1)}
_FUNCS = {np.sum: _f_sum, np.concatenate: _f_concatenate, np.reshape: _f_reshape, np.ravel: _f_ravel,
          np.shape: _f_shape, np.ndim: _f_ndim, np.size: _f_size, np.copy: _f_copy, np.transpose: _f_transpose,
          np.matmul: lambda a, b, **kw: _dispatch(_matmul, a, b, np.matmul) if not kw else _obj_call(np.matmul, (a, b), kw),
          np.dot: lambda a, b, out=None: _dispatch(_matmul, a, b, np.dot) if out is None else _obj_call(np.dot, (a, b), {"out": out}),
          np.stack: _f_stack}
