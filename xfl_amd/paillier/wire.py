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
# rows per encryption launch of a pipelined Paillier.encrypt (resident.encrypt_floats);
# $XHE_ENC_SUB overrides it (A/B measurement)
ENC_SUB = int(__import__("os").environ.get("XHE_ENC_SUB", 1 << 18))
_stage = {}           # (device, n2w) -> two pinned ([PIPE_CHUNK, n2w] words, [PIPE_CHUNK] bits), kept for the process
_copy_streams = {}    # device -> the pipeline's copy stream
_stage_lock = __import__("threading").Lock()
_TRACE = __import__("os").environ.get("XHE_PIPE_TRACE", "0") not in ("", "0")  # per-chunk timings on stderr  # one pipeline at a time uses the pinned buffers


def _copy_stream(dev):
    import torch
    s = _copy_streams.get(dev)
    if s is None:
        s = _copy_streams[dev] = torch.cuda.Stream(device=dev)
    return s


def encode_device(d, exps, shape, compression, dev):
    """encode_words of words held in HBM (an int32 tensor [count, n2w] on
    `dev`, written by kernels on the drop-in stream - e.g. an encryption that
    is still running), chunk by chunk: each chunk's D2H copy, on a copy
    stream, waits only for the encryption launches that write its rows (the
    readiness marks resident.encrypt_floats leaves on the tensor,
    `_xhe_ready`; else for everything queued so far) and lands in a pinned
    double buffer; the host lays the chunk out from the rows' own top words
    (xhe_wire_layout_part_rows: offsets from the previous chunk's end) and
    writes its rows (xhe_wire_rows) while the next chunk is encrypted and
    copied. The copy stream runs copies only - a kernel there would queue
    behind the encryption's blocks for CU slots. The payload is allocated at
    the size its elements could at most need (xhe_wire_begin) and cut to the
    real one at the end (finish, then an in-place shrink). The bytes equal
    encode_words(download(d), ...)."""
    import torch

    from .. import compat
    from . import resident
    count, n2w = int(d.shape[0]), int(d.shape[1])
    ex = np.ascontiguousarray(exps, dtype=np.int32).reshape(-1)
    shp = np.ascontiguousarray(shape, dtype=np.int64) if len(shape) else np.zeros(1, np.int64)
    L = nat.lib()
    off = np.empty(count + 1, dtype=np.int64)
    maxlen = ctypes.c_int64()
    # (count >= PIPE_MIN: the payload is above compat.RAW_FRAME_MIN, framed when compressed)
    framed = bool(compression)
    if count * 16 < compat.RAW_FRAME_MIN:
        raise ValueError("encode_device: below the pipeline's size (use encode_words)")
    nat.check(L.xhe_wire_begin(_vp(ex), count, n2w, _vp(shp), len(shape), int(framed), _vp(off),
                               ctypes.byref(maxlen), None, 0), "wire begin")
    out = nat.alloc_bytes(maxlen.value)
    optr = ctypes.c_void_p(ctypes.cast(out, ctypes.c_void_p).value)  # the address only (no reference)
    nat.check(L.xhe_wire_begin(_vp(ex), count, n2w, _vp(shp), len(shape), int(framed), _vp(off),
                               ctypes.byref(maxlen), optr, maxlen.value), "wire begin")
    marks = getattr(d, "_xhe_ready", None)
    if not marks or marks[-1][0] < count:
        with resident._On(dev):
            ev = torch.cuda.Event()
            ev.record(resident.stream(dev))
        marks = [(count, ev)]
    with _stage_lock:
        size = _pipeline(d, ex, count, n2w, dev, framed, off, maxlen, optr, marks)
    box = [out]
    del out  # the box holds the only reference: the cut is in place
    return nat.shrink_bytes(box, size)


def _pipeline(d, ex, count, n2w, dev, framed, off, maxlen, optr, marks):
    """encode_device's chunk loop (under _stage_lock: the pinned buffers are
    shared by every call); returns the payload's real size"""
    import torch
    L = nat.lib()
    rows = min(PIPE_CHUNK, count)
    st = _stage.get((dev, n2w))
    if st is None or st[0][0].shape[0] < rows:
        st = _stage[(dev, n2w)] = [(torch.empty((rows, n2w), dtype=torch.int32, pin_memory=True),
                                    torch.empty(rows, dtype=torch.int16, pin_memory=True)) for _ in range(2)]
    # the bit lengths the encryption computed behind each piece (else the host
    # reads them off the rows' top words)
    bits_d = getattr(d, "_xhe_bits", None)
    if bits_d is not None and bits_d.shape[0] != count:
        bits_d = None
    chunks = [(lo, min(count, lo + PIPE_CHUNK)) for lo in range(0, count, PIPE_CHUNK)]
    cs = _copy_stream(dev)
    evs = [None, None]
    waited = [0]  # marks the copy stream already waits for

    def issue(k):
        lo, hi = chunks[k]
        with torch.cuda.device(dev), torch.cuda.stream(cs):
            # every launch up to the one that writes row hi - 1 (launches on
            # two streams may finish out of order)
            while waited[0] < len(marks) and (waited[0] == 0 or marks[waited[0] - 1][0] < hi):
                cs.wait_event(marks[waited[0]][1])
                waited[0] += 1
            st[k % 2][0][:hi - lo].copy_(d[lo:hi], non_blocking=True)
            if bits_d is not None:
                st[k % 2][1][:hi - lo].copy_(bits_d[lo:hi], non_blocking=True)
            evs[k % 2] = torch.cuda.Event()
            evs[k % 2].record(cs)
    trace = _TRACE and []
    t0 = __import__("time").perf_counter()
    try:
        issue(0)
        for k, (lo, hi) in enumerate(chunks):
            if k + 1 < len(chunks):
                issue(k + 1)  # its buffer held chunk k - 1, written in the previous iteration
            evs[k % 2].synchronize()
            t1 = __import__("time").perf_counter()
            rp = ctypes.c_void_p(st[k % 2][0].data_ptr())
            if bits_d is not None:
                nat.check(L.xhe_wire_layout_part(ctypes.c_void_p(st[k % 2][1].data_ptr()), _vp(ex), lo, hi, count,
                                                 n2w, _vp(off)), "wire layout")
            else:
                nat.check(L.xhe_wire_layout_part_rows(rp, _vp(ex), lo, hi, count, n2w, _vp(off)), "wire layout")
            t2 = __import__("time").perf_counter()
            nat.check(L.xhe_wire_rows(rp, _vp(ex), lo, hi, count, n2w, _vp(off), int(framed), optr, maxlen.value),
                      "wire rows")
            if trace is not False:
                t3 = __import__("time").perf_counter()
                trace.append((k, round((t1 - t0) * 1e3, 2), round((t2 - t1) * 1e3, 2), round((t3 - t2) * 1e3, 2)))
        if trace:
            import sys
            print("pipeline (chunk, ready_ms, layout_ms, rows_ms):", trace, file=sys.stderr, flush=True)
    finally:
        cs.synchronize()  # no copy still landing in the shared pinned buffers (an error mid-way)
    size = ctypes.c_int64()
    nat.check(L.xhe_wire_finish(count, _vp(off), int(framed), optr, maxlen.value, ctypes.byref(size)), "wire finish")
    return size.value


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
