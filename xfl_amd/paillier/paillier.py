"""Paillier / PaillierCiphertext / RawCiphertext — drop-in for
python/common/crypto/paillier/paillier.py (same names, arguments, return
types and exceptions). Arithmetic runs on the GPU (xfl_amd.paillier.ops ->
include/xhe.h); results are bit-identical to the reference for the same keys
and obfuscation draws (tests/test_gpu_dropin.py).
"""
import pickle
import warnings
from typing import Optional, Union

import numpy as np

from .. import _native as nat
from . import ops, resident
from .context import PaillierContext
from .encoder import PaillierEncoder, int_to_float_gmpy
from .utils import MPZ, get_core_num  # noqa: F401  (re-exported like the reference)

_ST_ERR = {1: OverflowError, 2: ValueError}


class RawCiphertext:
    """paillier.py:39-42 — the pickled wire record (value, exp)."""

    def __init__(self, value, exp):
        self.value = value
        self.exp = exp


# Pickles must name the reference's module path so unmodified XFL peers can
# load what we emit (and we can load theirs): see xfl_amd/compat.py.
RawCiphertext.__module__ = "common.crypto.paillier.paillier"


def _is_scalar(x):
    return isinstance(x, (int, float)) and not isinstance(x, bool) or isinstance(x, bool)


class PaillierCiphertext(object):
    """paillier.py:45-232

    Ciphertext + ciphertext is DEFERRED: the result records its two operands
    and its exponent (min of theirs, paillier.py:106-123) and computes the
    residue on first use. The folded value of any tree of such additions is
    prod c_i^(2^(e_i - e_min)) mod n^2 in any order, so a
    chain of n additions (pandas groupby sum, np.sum over object arrays,
    Python sum()) costs n O(1) Python steps and ONE segmented-product kernel
    call when the result is read, instead of n device round trips. Reading
    raw_ciphertext, serializing, decrypting or any batched operation
    materializes (materialize() does a whole array in one call).
    """

    __slots__ = ("_PaillierCiphertext__context", "_PaillierCiphertext__c", "_PaillierCiphertext__exp", "_parts")

    def __init__(self, context: PaillierContext, raw_ciphertext: MPZ, exponent: int) -> None:
        self.__context = context
        self.__c = None if raw_ciphertext is None else int(raw_ciphertext)
        self.__exp = int(exponent)
        self._parts = None  # (a, b) while this is a deferred a + b

    @classmethod
    def _deferred_sum(cls, a, b):
        ct = cls(a.context, None, min(a.exponent, b.exponent))
        ct._parts = (a, b)
        return ct

    def _is_deferred(self):
        return self.__c is None

    def _set_raw(self, raw):
        self.__c = int(raw)
        self._parts = None

    @property
    def context(self):
        return self.__context

    @property
    def raw_ciphertext(self):
        if self.__c is None:
            materialize([self])
        return self.__c

    @property
    def exponent(self):
        return self.__exp

    def serialize(self, compression: bool = True) -> bytes:
        from ..compat import compress, dumps
        out = dumps(RawCiphertext(self.raw_ciphertext, self.__exp))
        return compress(out) if compression else out

    @classmethod
    def deserialize_from(cls, context: PaillierContext, data: bytes, compression: bool = True):
        from ..compat import decompress, loads
        if compression:
            data = decompress(data)
        r = loads(data)
        return PaillierCiphertext(context, int(r.value), r.exp)

    def _decrease_exponent_to(self, new_exponent: int):
        """paillier.py:79-86"""
        scalar = 1 << (self.__exp - new_exponent)
        return ops.raw_mul(self.__context, [self.raw_ciphertext], [scalar])[0]

    def __add__(self, other):
        """paillier.py:88-104 (no obfuscation when adding a scalar)."""
        if isinstance(other, PaillierCiphertext):
            return self._add_encrypted(other)
        elif isinstance(other, (int, float)):
            ciphertext = Paillier.encrypt(self.context, other, precision=None, max_exponent=None, obfuscation=False)
            return self._add_encrypted(ciphertext)
        else:
            raise TypeError(f"Adding data of type {type(other)} not supported.")

    def _add_encrypted(self, other):
        """paillier.py:106-123 (deferred: see the class docstring)"""
        if self.context is not other.context and self.context.to_public() != other.context.to_public():
            raise ValueError("Adding two ciphertext with different keys.")
        return PaillierCiphertext._deferred_sum(self, other)

    def __radd__(self, other):
        return self.__add__(other)

    def __sub__(self, other):
        return self.__add__(other * (-1))

    def __rsub__(self, other):
        return ((-1) * self).__add__(other)

    def __mul__(self, scalar: Union[int, float]):
        """paillier.py:134-145"""
        if isinstance(scalar, PaillierCiphertext):
            raise TypeError("Cannot multiply one ciphertext with another ciphertext, try multiply a scalar.")
        exponent = PaillierEncoder.cal_exponent(scalar, precision=None)
        encoded_scalar = PaillierEncoder.encode_single(self.context, scalar, exponent)
        raw = ops.raw_mul(self.__context, [self.raw_ciphertext], [encoded_scalar])[0]
        return PaillierCiphertext(self.context, raw, exponent + self.exponent)

    def __rmul__(self, scalar: Union[int, float]):
        return self.__mul__(scalar)

    def __truediv__(self, scalar: Union[int, float]):
        return self.__mul__(1 / scalar)

    def obfuscate(self):
        """paillier.py:189-232 (fresh device-drawn a / r)."""
        self._set_raw(ops.obfuscate(self.__context, [self.raw_ciphertext])[0])
        return self


def materialize(cts):
    """Compute every deferred sum among `cts` with one segmented product per
    key: each deferred ciphertext becomes the product of the leaves of its
    addition tree, aligned to its exponent (paillier.py:79-86,106-123)."""
    pending = [c for c in cts if isinstance(c, PaillierCiphertext) and c._is_deferred()]
    if not pending:
        return
    by_ctx = {}
    seen = set()
    for c in pending:
        if id(c) not in seen:
            seen.add(id(c))
            by_ctx.setdefault(id(c.context), []).append(c)
    for group in by_ctx.values():
        raws, exps, seg = [], [], [0]
        gaps = {}  # leaves whose path crosses a negative-branch alignment (ops.gap_power)
        dneg = ops.gap_threshold(group[0].context)
        for root in group:
            stack = [(root, ())]
            while stack:  # iterative: addition chains can be 10^5 deep
                node, bigs = stack.pop()
                if node._is_deferred():
                    for part in node._parts:
                        s = part.exponent - node.exponent  # the shift _add_encrypted aligns `part` by
                        stack.append((part, bigs + (s,) if s >= dneg else bigs))
                else:
                    if bigs:
                        gaps[len(raws)] = ops.gap_power(node.context, node.exponent - root.exponent, bigs)
                    raws.append(node.raw_ciphertext)
                    exps.append(node.exponent)
            seg.append(len(raws))
        r, e = ops.segment_sums(group[0].context, raws, exps, seg, gap_powers=gaps)
        for root, rv, ev in zip(group, r, e):
            assert int(ev) == root.exponent
            root._set_raw(rv)


def raws_of(cts):
    """raw ciphertexts of a sequence, deferred sums materialized in one batch"""
    materialize(cts)
    return [c.raw_ciphertext for c in cts]


def _encode_ints(context, xs, precision, max_exponent):
    """Reference per-element encode for integer elements (encoder.py:29-54)."""
    ms, es = [], []
    for x in xs:
        e = PaillierEncoder.cal_exponent(x, precision)
        if max_exponent is not None:
            e = min(e, max_exponent)
        ms.append(int(PaillierEncoder.encode_single(context, x, e)))
        es.append(int(e))
    return ms, es


class Paillier(object):
    """paillier.py:235-431"""

    @staticmethod
    def context(key_bit_size: int = 2048, djn_on: bool = False):
        return PaillierContext.generate(key_bit_size, djn_on)

    @staticmethod
    def context_from(data: bytes):
        return PaillierContext.deserialize_from(data)

    @staticmethod
    def serialize(data: Union[np.ndarray, PaillierCiphertext], compression: bool = True) -> bytes:
        """paillier.py:244-258: the pickle of an ndarray[object] of
        RawCiphertext, written natively from the flat words (wire.hpp)."""
        from ..compat import compress, dumps
        from . import wire
        from .array import PaillierArray, _check_no_na
        if isinstance(data, PaillierCiphertext):
            return data.serialize(compression)
        if isinstance(data, PaillierArray):
            _check_no_na(data)
            st = data._st
            if st.h is None and st.d is not None and data.size >= wire.PIPE_MIN:
                # words only in HBM (a fresh encryption or operation result):
                # laid out from their bit lengths, downloaded and encoded in
                # overlapping chunks
                dev = st.d.device.index
                return wire.encode_device(data._dw(dev), data.exponents, data.shape, compression, dev)
            return wire.encode_words(data.words, data.exponents, data.shape, compression=compression)
        if isinstance(data, np.ndarray) and data.dtype == object:
            flat = list(data.reshape(-1))
            materialize(flat)
            if flat and all(isinstance(x, PaillierCiphertext) for x in flat):
                raws = [x.raw_ciphertext for x in flat]
                ctx = flat[0].context
                bits = ctx.n_square.bit_length() if ctx is not None else max(r.bit_length() for r in raws)
                n2w = max(1, (bits + 31) // 32)
                ct = nat.ints_to_words(raws, n2w) if raws else np.zeros((0, n2w), np.uint32)
                return wire.encode_words(ct, [x.exponent for x in flat], data.shape, compression=compression)

        def f(x):
            return RawCiphertext(x.raw_ciphertext, x.exponent)

        out = dumps(np.vectorize(f)(data))
        return compress(out) if compression else out

    @staticmethod
    def ciphertext_from(context: PaillierContext, data: bytes, compression: bool = True):
        """paillier.py:260-271 -> PaillierArray (context may be None, as in
        label_trainer.py:258; pass the key to decrypt)."""
        from ..compat import decompress, loads
        from .array import PaillierArray
        if compression:
            data = decompress(data)
        try:  # native decode of the ciphertext-array format, straight into words
            from . import wire
            w, e, shape = wire.decode_words(data, ops.n2w_of(context) if context is not None else None)
            return PaillierArray.from_buffers(context, w, e, shape)
        except ValueError:
            pass
        unpickled = loads(data)

        def f(x):
            return PaillierCiphertext(context, int(x.value), x.exp)

        return PaillierArray(np.vectorize(f, otypes=[PaillierCiphertext])(unpickled), context=context)

    @classmethod
    def encrypt(cls, context: PaillierContext, data: Union[int, float, np.ndarray], precision: Optional[int] = None,
                max_exponent: Optional[int] = None, obfuscation: bool = True,
                num_cores: int = -1) -> Union[PaillierCiphertext, np.ndarray]:
        """paillier.py:289-339. Arrays come back as a PaillierArray (flat
        words + exponents, ciphertext objects on element access); num_cores
        spreads the elements over GPUs (PaillierContext.shard_devices) where
        the reference spreads them over processes."""
        from .array import PaillierArray
        if isinstance(data, np.ndarray):
            shape = data.shape
            flat = data.reshape(-1)
            n = flat.shape[0]
            # ciphertext words + exponent + the staged plaintext per element
            dev = resident.device_for(context, num_cores, n, 4 * ops.n2w_of(context) + 16) if n else None
            if flat.dtype.kind == "f":
                if dev is not None:  # results stay in HBM (resident.py)
                    if obfuscation:
                        context.note_encrypt_volume(n)
                    d, e, st = resident.encrypt_floats(context.device_key(dev), flat, precision, max_exponent,
                                                       obfuscation)
                    Paillier._raise_status(st)
                    return PaillierArray.from_device(context, d, e, shape)
                w, e, st = ops.encrypt_floats_words(context, flat, precision, max_exponent, obfuscation, num_cores)
                Paillier._raise_status(st)
                return PaillierArray.from_buffers(context, w, e, shape)
            nw = ops.nw_of(context)
            mw = np.zeros((n, nw), dtype=np.uint32)
            exps = np.zeros(n, dtype=np.int32)
            fl_idx, int_idx = [], []
            if flat.dtype.kind in "iub":
                int_idx = range(n)
                if dev is not None:
                    ms, es = _encode_ints(context, flat.tolist(), precision, max_exponent)
                    if obfuscation:
                        context.note_encrypt_volume(n)
                    d = resident.encrypt_encoded(context.device_key(dev), nat.ints_to_words(ms, nw), obfuscation)
                    return PaillierArray.from_device(context, d, np.asarray(es, dtype=np.int32), shape)
            else:
                for i, x in enumerate(flat):
                    if isinstance(x, (float, np.floating)):
                        fl_idx.append(i)
                    elif isinstance(x, (int, np.integer)):
                        int_idx.append(i)
                    else:
                        PaillierEncoder.cal_exponent(x, precision)  # raises TypeError like the reference
                        raise TypeError(f"Unsupported data type {type(x)}")
            words = np.empty((n, ops.n2w_of(context)), dtype=np.uint32)
            if len(fl_idx):
                fi = np.asarray(fl_idx, dtype=np.int64)
                w, e, st = ops.encrypt_floats_words(context, np.array([float(flat[i]) for i in fl_idx]), precision,
                                                    max_exponent, obfuscation, num_cores)
                Paillier._raise_status(st)
                words[fi] = w
                exps[fi] = e
            if len(int_idx):
                ii = np.asarray(int_idx, dtype=np.int64)
                ms, es = _encode_ints(context, [flat[i] for i in int_idx], precision, max_exponent)
                words[ii] = ops.encrypt_encoded_words(context, nat.ints_to_words(ms, nw), obfuscation, num_cores)
                exps[ii] = es
            return PaillierArray.from_buffers(context, words, exps, shape)
        elif isinstance(data, (int, float)):
            if isinstance(data, float):
                r, e, st = ops.encrypt_floats(context, np.array([data]), precision, max_exponent, obfuscation)
                Paillier._raise_status(st)
                return PaillierCiphertext(context, r[0], int(e[0]))
            ms, es = _encode_ints(context, [data], precision, max_exponent)
            return PaillierCiphertext(context, ops.encrypt_encoded(context, ms, obfuscation)[0], es[0])
        else:
            raise TypeError(f"Unsupported data type {type(data)}, accepted types are 'np.ndarray', 'int', 'float'.")

    @staticmethod
    def _raise_status(st):
        bad = np.nonzero(st)[0]
        if bad.size:
            code = int(st[bad[0]])
            if code == 2:
                raise ValueError("cannot convert float NaN to integer / negative shift count")
            raise OverflowError("cannot convert float infinity to integer / int too large to convert to float")

    @staticmethod
    def _decrypt_single(data: PaillierCiphertext, context: PaillierContext):
        """paillier.py:341-368 (non-ciphertexts pass through)."""
        if not isinstance(data, PaillierCiphertext):
            return data
        m = ops.decrypt_ints(context, [data.raw_ciphertext])[0]
        return PaillierEncoder.decode_single(context, m, data.exponent)

    @classmethod
    def decrypt(cls, context: PaillierContext, data: Union[PaillierCiphertext, np.ndarray], dtype: str = 'float',
                num_cores: int = -1, out_origin: bool = False):
        """paillier.py:370-417"""
        from .array import SMALL, PaillierArray
        if not context.is_private():
            raise TypeError("Try to decrypt a paillier ciphertext by a public key.")
        if isinstance(data, PaillierArray):
            if data._has_na():  # missing entries pass through as NaN (paillier.py:344-345: non-ciphertexts)
                return cls.decrypt(context, data.astype(object), dtype, num_cores, out_origin)
            arr = data._aligned_words(ops.n2w_of(context))
            dev = resident.device_for(context, num_cores)
            if arr.size and (arr._resident_on(dev) or (dev is not None and arr.size <= SMALL)):
                # in HBM (or small enough to upload): only the results come back
                dk = context.device_key(dev)
                if not out_origin and dtype == 'float':
                    _, f32, st = resident.decrypt_decode(dk, arr._dw(dev), arr.exponents)
                    if np.any(st != 0):
                        raise OverflowError("Overflow detected during decoding encrypted number.")
                    return f32.reshape(arr.shape)
                ms = nat.words_to_ints(resident.decrypt(dk, arr._dw(dev)))
                vals = [PaillierEncoder.decode_single(context, m, int(e)) for m, e in zip(ms, arr.exponents.tolist())]
                out = np.empty(len(vals), dtype=object)
                out[:] = vals
                return _finish_decrypt(out.reshape(arr.shape), dtype, out_origin)
            if not out_origin and dtype == 'float':
                # decrypt + decode + float32 on the device, straight from the words
                _, f32, st = ops.decrypt_decode_words(context, arr.words, arr.exponents, num_cores)
                if np.any(st != 0):
                    raise OverflowError("Overflow detected during decoding encrypted number.")
                return f32.reshape(arr.shape)
            ms = nat.words_to_ints(ops.decrypt_words(context, arr.words, num_cores)) if arr.size else []
            vals = [PaillierEncoder.decode_single(context, m, int(e)) for m, e in zip(ms, arr.exponents.tolist())]
            out = np.empty(len(vals), dtype=object)
            out[:] = vals
            return _finish_decrypt(out.reshape(arr.shape), dtype, out_origin)
        if isinstance(data, np.ndarray):
            shape = data.shape
            flat = data.reshape(-1)
            idx = [i for i, x in enumerate(flat) if isinstance(x, PaillierCiphertext)]
            if not out_origin and dtype == 'float' and len(idx) == len(flat) and len(flat) > 0:
                _, f32, st = ops.decrypt_float32(context, raws_of(list(flat)), [x.exponent for x in flat])
                if np.any(st != 0):
                    raise OverflowError("Overflow detected during decoding encrypted number.")
                return f32.reshape(shape)
            vals = list(flat)
            ms = ops.decrypt_ints(context, raws_of([flat[i] for i in idx]))
            for i, m in zip(idx, ms):
                vals[i] = PaillierEncoder.decode_single(context, m, flat[i].exponent)
            out = np.empty(len(vals), dtype=object)
            out[:] = vals
            return _finish_decrypt(out.reshape(shape), dtype, out_origin)
        elif isinstance(data, PaillierCiphertext):
            out = cls._decrypt_single(data, context)
            if not out_origin:
                if 'float' in dtype:
                    out = float(out) if isinstance(out, float) else int_to_float_gmpy(out)
                elif 'int' in dtype:
                    out = int(out)
                else:
                    warnings.warn(f"dtype {dtype} not supported.")
                    out = float(out) if isinstance(out, float) else int_to_float_gmpy(out)
            return out
        else:
            raise TypeError(f"Unsupported data type {type(data)}, accepted types are 'np.ndarray', "
                            "'PaillierCiphertext'.")

    @classmethod
    def obfuscate(cls, ciphertext: Union[PaillierCiphertext, np.ndarray]):
        """paillier.py:419-431: re-randomises the ciphertexts in place (the
        reference calls c.obfuscate() on each element) and returns them."""
        from .array import PaillierArray
        if isinstance(ciphertext, PaillierArray):
            ctx = ciphertext.context
            if ciphertext.size:
                if ctx is None:
                    raise ValueError("ciphertext array without a context")
                ciphertext._obfuscate_in_place()
            return ciphertext
        if isinstance(ciphertext, np.ndarray):
            flat = ciphertext.reshape(-1)
            if not all(isinstance(c, PaillierCiphertext) for c in flat):
                raise TypeError("Unsupported raw ciphertext type")
            if len(flat):
                ctx = flat[0].context
                raws = ops.obfuscate(ctx, raws_of(list(flat)))
                for c, r in zip(flat, raws):
                    c._set_raw(r)
            return ciphertext
        elif isinstance(ciphertext, PaillierCiphertext):
            return ciphertext.obfuscate()
        else:
            raise TypeError(f"Unsupported raw ciphertext type {type(ciphertext)}")


def _finish_decrypt(out, dtype, out_origin):
    """paillier.py:396-414: the array's dtype conversion after decode."""
    if out_origin:
        return out
    if dtype == 'float':
        return _astype_f32(out)
    if dtype == 'int':
        return out.astype(np.int32)
    warnings.warn(f"dtype {dtype} not supported.")
    return _astype_f32(out)


def _astype_f32(obj_arr):
    """astype(np.float32) of decode outputs: floats directly, ints through the
    gmpy2 mpz->float conversion (truncating) like the reference's mpz objects."""
    flat = obj_arr.reshape(-1)
    vals = np.empty(len(flat), dtype=np.float64)
    for i, v in enumerate(flat):
        if isinstance(v, float):
            vals[i] = v
        elif isinstance(v, int):
            vals[i] = int_to_float_gmpy(v)
        else:
            vals[i] = float(v)
    with np.errstate(over="ignore"):
        return vals.astype(np.float32).reshape(obj_arr.shape)
