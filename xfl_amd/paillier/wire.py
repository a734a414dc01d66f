"""Native wire codec for ciphertext arrays (xhe_wire_encode / xhe_wire_decode,
include/xhe.h): Paillier.serialize / ciphertext_from (paillier.py:244-271)
without a Python pickle round of one RawCiphertext object per element. The
bytes are a standard pickle of np.ndarray[object] of RawCiphertext, loadable
by XFL peers (numpy 1.x or 2.x); decoding accepts CPython's pickles of that
graph, including the reference's gmpy2 values. Host-only: no device needed.
"""
import ctypes

import numpy as np

from .. import _native as nat

_MAX_WORDS = 512  # n^2 of an 8192-bit key, the largest device key size (context.SUPPORTED_DEVICE_BITS)


def _vp(a):
    return ctypes.c_void_p(a.ctypes.data)


def encode(raws, exps, shape, n2w):
    """pickle bytes of the ndarray (shape) of RawCiphertext(raws[i], exps[i])."""
    ct = nat.ints_to_words(raws, n2w) if len(raws) else np.zeros((0, n2w), np.uint32)
    return encode_words(ct, exps, shape)


def encode_words(ct, exps, shape):
    """pickle bytes of the ndarray (shape) of RawCiphertext from flat buffers:
    ct uint32 [count, n2w], exps int32 [count]."""
    ct = np.ascontiguousarray(ct, dtype=np.uint32)
    count, n2w = ct.shape
    if count == 0:
        ct = np.zeros((1, n2w), np.uint32)
    ex = np.ascontiguousarray(exps, dtype=np.int32) if count else np.zeros(1, np.int32)
    shp = np.ascontiguousarray(shape, dtype=np.int64) if len(shape) else np.zeros(1, np.int64)
    L = nat.lib()
    need = ctypes.c_int64()
    rc = L.xhe_wire_encode(_vp(ct), _vp(ex), count, n2w, _vp(shp), len(shape), None, 0, ctypes.byref(need))
    if rc != nat.XHE_EOVERFLOW:
        nat.check(rc, "wire encode")
    # written straight into the bytes object handed back (no staging copy of
    # the ~0.5 KB/ciphertext payload); nothing else references it yet
    out = bytes(need.value)  # > 100 bytes (header): never a shared singleton
    ptr = ctypes.cast(out, ctypes.c_void_p)
    nat.advise_huge(ptr.value, need.value)
    rc = L.xhe_wire_encode(_vp(ct), _vp(ex), count, n2w, _vp(shp), len(shape), ptr, need.value,
                           ctypes.byref(need))
    nat.check(rc, "wire encode")
    return out


def decode(data, n2w=None):
    """(raw ints, exponents, shape) of a ciphertext-array pickle; raises
    ValueError when the bytes are not that format."""
    ct, ex, shape = _decode(data, n2w or _MAX_WORDS)
    return (nat.words_to_ints(ct) if ct.shape[0] else []), ex, shape


# word widths tried for a payload decoded without a context: n^2 of the
# device key sizes (context.SUPPORTED_DEVICE_BITS), narrowest first
_WIDTHS = (128, 192, 256, 512)


def decode_words(data, n2w=None):
    """(uint32 words [count, n2w], int32 exponents, shape) of a
    ciphertext-array pickle. Without n2w the narrowest device width that
    holds every value is used. Raises ValueError when the bytes are not that
    format."""
    if n2w is not None:
        return _decode(data, n2w)
    err = None
    for w in _WIDTHS:
        try:
            return _decode(data, w)
        except ValueError as e:  # "value too large" -> next width; anything else is final
            err = e
            if "too large" not in str(e):
                raise
    raise err


def _decode(data, n2w):
    L = nat.lib()
    buf = np.frombuffer(data, dtype=np.uint8)
    count = ctypes.c_int64()
    ndim = ctypes.c_int()
    shape = np.zeros(8, dtype=np.int64)
    cap = max(1, len(data) // (4 * n2w) + 16)
    for _ in range(2):
        ct = nat.empty((cap, n2w), np.uint32)
        ex = np.empty(cap, dtype=np.int32)
        rc = L.xhe_wire_decode(_vp(buf), len(data), n2w, _vp(ct), _vp(ex), cap, ctypes.byref(count), _vp(shape),
                               ctypes.byref(ndim))
        if rc != nat.XHE_EOVERFLOW:
            break
        cap = count.value
    if rc != nat.XHE_OK:
        raise ValueError(nat.lib().xhe_last_error().decode(errors="replace"))
    n = count.value
    return ct[:n], ex[:n], tuple(int(s) for s in shape[:ndim.value])
