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


def encode_words(ct, exps, shape, compression=False):
    """pickle bytes of the ndarray (shape) of RawCiphertext from flat buffers:
    ct uint32 [count, n2w], exps int32 [count]. compression=True: what
    compat.compress makes of those bytes (paillier.py:244-258) - from
    compat.RAW_FRAME_MIN up the zstd raw-block frame, written in one pass
    (xhe_wire_encode_frame: no intermediate pickle buffer)."""
    ct = np.ascontiguousarray(ct, dtype=np.uint32)
    count, n2w = ct.shape
    if count == 0:
        ct = np.zeros((1, n2w), np.uint32)
    ex = np.ascontiguousarray(exps, dtype=np.int32) if count else np.zeros(1, np.int32)
    shp = np.ascontiguousarray(shape, dtype=np.int64) if len(shape) else np.zeros(1, np.int64)
    L = nat.lib()
    need = ctypes.c_int64()

    def enc(framed, out, cap):
        return L.xhe_wire_encode_frame(_vp(ct), _vp(ex), count, n2w, _vp(shp), len(shape), int(framed), out, cap,
                                       ctypes.byref(need))
    rc = enc(False, None, 0)
    if rc != nat.XHE_EOVERFLOW:
        nat.check(rc, "wire encode")
    from .. import compat
    framed = compression and need.value >= compat.RAW_FRAME_MIN
    if compression and not framed:  # small payloads: libzstd level 3, as before
        return compat.compress(encode_words(ct[:count], ex[:count], shape))
    if framed:
        rc = enc(True, None, 0)
        if rc != nat.XHE_EOVERFLOW:
            nat.check(rc, "wire encode")
    # written straight into the bytes object handed back (every byte of it),
    # from the process heap when large (nat.alloc_bytes)
    out = nat.alloc_bytes(need.value)
    nat.check(enc(framed, ctypes.cast(out, ctypes.c_void_p), need.value), "wire encode")
    return out


PIPE_MIN = 1 << 16    # device arrays from this many rows serialize through the pipeline below
PIPE_CHUNK = 1 << 17  # rows per D2H chunk (64 MB at 2048 bits)
_stage = {}           # (device, n2w) -> two pinned [PIPE_CHUNK, n2w] buffers, kept for the process


def encode_device(d, exps, shape, compression, dev):
    """encode_words of words held in HBM (an int32 tensor [count, n2w] on
    `dev`, written by kernels on the drop-in stream - e.g. an encryption that
    is still running): the bit length of every row is computed on the device
    (xhe_row_bits) and comes down first, so the payload is laid out and
    allocated before the words (xhe_wire_layout); then the rows come down in
    chunks into a pinned double buffer, the D2H copy of chunk k + 1 running
    while the host threads encode chunk k (xhe_wire_rows). The bytes equal
    encode_words(download(d), ...)."""
    import torch

    from .. import compat
    from . import resident
    count, n2w = int(d.shape[0]), int(d.shape[1])
    ex = np.ascontiguousarray(exps, dtype=np.int32).reshape(-1)
    shp = np.ascontiguousarray(shape, dtype=np.int64) if len(shape) else np.zeros(1, np.int64)
    L = nat.lib()
    with resident._On(dev):
        bits_d = torch.empty(count, dtype=torch.int16, device=f"cuda:{dev}")
    nat.check(L.xhe_row_bits(resident._dp(d), count, n2w, resident._dp(bits_d), resident._sp(dev)), "row bits")
    bits = resident.download(bits_d, np.int16)  # (waits for the kernels that write d)
    offs = np.empty(count + 1, dtype=np.int64)
    need = ctypes.c_int64()

    def lay(framed, out, cap):
        nat.check(L.xhe_wire_layout(_vp(bits), _vp(ex), count, n2w, _vp(shp), len(shape), int(framed), _vp(offs), out,
                                    cap, ctypes.byref(need)), "wire layout")
    lay(False, None, 0)
    framed = compression and need.value >= compat.RAW_FRAME_MIN
    if compression and not framed:
        return encode_words(resident.download(d), ex, shape, compression=True)
    if framed:
        lay(True, None, 0)
    out = nat.alloc_bytes(need.value)
    optr = ctypes.cast(out, ctypes.c_void_p)
    lay(framed, optr, need.value)
    rows = min(PIPE_CHUNK, count)
    bufs = _stage.get((dev, n2w))
    if bufs is None or bufs[0].shape[0] < rows:
        bufs = _stage[(dev, n2w)] = [torch.empty((rows, n2w), dtype=torch.int32, pin_memory=True) for _ in range(2)]
    chunks = [(lo, min(count, lo + PIPE_CHUNK)) for lo in range(0, count, PIPE_CHUNK)]
    s = resident.stream(dev)
    evs = [None, None]

    def issue(k):
        lo, hi = chunks[k]
        with resident._On(dev):
            bufs[k % 2][:hi - lo].copy_(d[lo:hi], non_blocking=True)
            evs[k % 2] = torch.cuda.Event()
            evs[k % 2].record(s)
    issue(0)
    for k, (lo, hi) in enumerate(chunks):
        if k + 1 < len(chunks):
            issue(k + 1)  # its buffer held chunk k - 1, encoded in the previous iteration
        evs[k % 2].synchronize()
        nat.check(L.xhe_wire_rows(ctypes.c_void_p(bufs[k % 2].data_ptr()), _vp(ex), lo, hi, count, n2w, _vp(offs),
                                  int(framed), optr, need.value), "wire rows")
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
