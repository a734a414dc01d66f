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
    count = len(raws)
    ct = nat.ints_to_words(raws, n2w) if count else np.zeros((1, n2w), np.uint32)
    ex = np.ascontiguousarray(exps, dtype=np.int32) if count else np.zeros(1, np.int32)
    shp = np.ascontiguousarray(shape, dtype=np.int64) if len(shape) else np.zeros(1, np.int64)
    L = nat.lib()
    need = ctypes.c_int64()
    cap = 256 + count * (4 * n2w + 24)
    out = np.empty(cap, dtype=np.uint8)
    rc = L.xhe_wire_encode(_vp(ct), _vp(ex), count, n2w, _vp(shp), len(shape), _vp(out), cap, ctypes.byref(need))
    if rc == nat.XHE_EOVERFLOW:
        out = np.empty(need.value, dtype=np.uint8)
        rc = L.xhe_wire_encode(_vp(ct), _vp(ex), count, n2w, _vp(shp), len(shape), _vp(out), need.value,
                               ctypes.byref(need))
    nat.check(rc, "wire encode")
    return out[:need.value].tobytes()


def decode(data, n2w=None):
    """(raw ints, exponents, shape) of a ciphertext-array pickle; raises
    ValueError when the bytes are not that format."""
    n2w = n2w or _MAX_WORDS
    L = nat.lib()
    buf = np.frombuffer(data, dtype=np.uint8)
    count = ctypes.c_int64()
    ndim = ctypes.c_int()
    shape = np.zeros(8, dtype=np.int64)
    cap = max(1, len(data) // (4 * n2w) + 16)
    for _ in range(2):
        ct = np.empty((cap, n2w), dtype=np.uint32)
        ex = np.empty(cap, dtype=np.int32)
        rc = L.xhe_wire_decode(_vp(buf), len(data), n2w, _vp(ct), _vp(ex), cap, ctypes.byref(count), _vp(shape),
                               ctypes.byref(ndim))
        if rc != nat.XHE_EOVERFLOW:
            break
        cap = count.value
    if rc != nat.XHE_OK:
        raise ValueError(nat.lib().xhe_last_error().decode(errors="replace"))
    n = count.value
    return nat.words_to_ints(ct[:n]) if n else [], ex[:n], tuple(int(s) for s in shape[:ndim.value])
