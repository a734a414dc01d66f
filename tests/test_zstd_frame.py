"""The zstd framing of Paillier.serialize(compression=True) (paillier.py:244-271):
large payloads become one frame of raw blocks (xhe_zstd_raw_frame), which the
system libzstd - the decoder the reference's zstd.decompress wraps - must read
back bit-exactly; small ones stay libzstd level-3 frames. Host only (CPU)."""
import ctypes

import numpy as np
import pytest

from xfl_amd import _native as nat
from xfl_amd import compat

BLOCK = 1 << 17


def libzstd_decompress(frame):
    L = compat._lib()
    size = L.ZSTD_getFrameContentSize(frame, len(frame))
    assert size < (1 << 63), "frame must carry its content size"
    dst = ctypes.create_string_buffer(max(int(size), 1))
    n = L.ZSTD_decompress(dst, int(size), frame, len(frame))
    assert not L.ZSTD_isError(n), "libzstd rejected the frame"
    return dst.raw[:n]


@pytest.mark.parametrize("n", [compat.RAW_FRAME_MIN, 8 * BLOCK + 1, 64 * BLOCK, (9 << 20) + 12345])
def test_raw_frame_reads_back_through_libzstd(n):
    data = np.random.default_rng(n).integers(0, 256, n, dtype=np.uint8).tobytes()
    frame = compat.compress(data)
    assert len(frame) == nat.lib().xhe_zstd_raw_frame_size(n) == 14 + n + 3 * (-(-n // BLOCK))
    assert frame[:4] == b"\x28\xb5\x2f\xfd"
    assert libzstd_decompress(frame) == data      # any zstd decoder
    assert compat.decompress(frame) == data       # the parallel raw path
    assert compat._raw_extract(frame) == data


def test_small_payloads_stay_libzstd_frames():
    data = b"RawCiphertext" * 1000
    frame = compat.compress(data)
    assert len(frame) < len(data) // 10           # really compressed
    assert compat._raw_extract(frame) is None      # not raw blocks: libzstd path
    assert compat.decompress(frame) == data


def test_libzstd_frames_take_the_libzstd_path():
    data = (b"\x00" * 100 + bytes(range(256))) * 8000   # > RAW_FRAME_MIN, compressible
    L = compat._lib()
    cap = L.ZSTD_compressBound(len(data))
    dst = ctypes.create_string_buffer(cap)
    k = L.ZSTD_compress(dst, cap, data, len(data), 3)
    frame = dst.raw[:k]
    assert compat._raw_extract(frame) is None
    assert compat.decompress(frame) == data


def test_raw_extract_rejects_damaged_frames():
    data = np.random.default_rng(1).integers(0, 256, 3 * BLOCK + 7, dtype=np.uint8).tobytes()
    frame = bytearray(compat.compress(data))
    L = nat.lib()
    n = ctypes.c_int64()
    for bad in (frame[:-1], frame + b"\x00", frame[:20]):
        bad = bytes(bad)
        assert L.xhe_zstd_raw_extract(bad, len(bad), None, 0, ctypes.byref(n)) == nat.XHE_ENOTSUP
    wrong_size = bytearray(frame)
    wrong_size[6] ^= 1                             # content size no longer matches the blocks
    wrong_size = bytes(wrong_size)
    assert L.xhe_zstd_raw_extract(wrong_size, len(wrong_size), None, 0, ctypes.byref(n)) == nat.XHE_ENOTSUP
    checksum = bytearray(frame)
    checksum[4] |= 0x04                            # content checksum flag: left to libzstd
    checksum = bytes(checksum)
    assert L.xhe_zstd_raw_extract(checksum, len(checksum), None, 0, ctypes.byref(n)) == nat.XHE_ENOTSUP
    good = bytes(frame)
    assert L.xhe_zstd_raw_extract(good, len(good), None, 0, ctypes.byref(n)) == nat.XHE_EOVERFLOW
    assert n.value == len(data)


def test_serialize_compressed_roundtrip_large_array():
    """Paillier.serialize(compression=True) of a ciphertext array above the
    threshold -> ciphertext_from(compression=True) gives the same words."""
    from xfl_amd.paillier import Paillier
    from xfl_amd.paillier.array import PaillierArray
    count, n2w = 4096, 128
    w = np.random.default_rng(2).integers(0, 1 << 32, (count, n2w), dtype=np.uint64).astype(np.uint32)
    w[:, -1] &= 0x7FFFFFFF
    e = np.random.default_rng(3).integers(-60, 0, count).astype(np.int32)
    arr = PaillierArray.from_buffers(None, w, e, (count,))
    blob = Paillier.serialize(arr, compression=True)
    assert len(blob) > compat.RAW_FRAME_MIN
    plain = libzstd_decompress(blob)
    assert plain == Paillier.serialize(arr, compression=False)
    back = Paillier.ciphertext_from(None, blob, compression=True)
    assert np.array_equal(back.words, w) and np.array_equal(back.exponents, e)


@pytest.mark.parametrize("framed", [False, True])
def test_incremental_layout_equals_one_pass(framed):
    """The serialize pipeline's range-by-range layout (xhe_wire_begin /
    layout_part / rows / finish over a payload allocated at the largest size
    the elements could need, then cut in place by shrink_bytes) gives the
    bytes of the one-pass writer (xhe_wire_encode_frame), for ranges that
    cross APPENDS batches and zstd block borders."""
    from xfl_amd.paillier import wire
    rng = np.random.default_rng(8)
    count, n2w = 5003, 128
    ct = rng.integers(0, 2 ** 32, (count, n2w), dtype=np.uint64).astype(np.uint32)
    ct[:, -1] >>= rng.integers(0, 32, count).astype(np.uint32)  # ragged bit lengths
    ct[7] = 0
    ex = rng.integers(-3, 400, count).astype(np.int32)
    shape = (count,)
    want = wire.encode_words(ct, ex, shape)
    if framed:
        want = compat.compress(want) if len(want) < compat.RAW_FRAME_MIN else wire.encode_words(ct, ex, shape, True)
    L = nat.lib()
    vp = lambda a: ctypes.c_void_p(a.ctypes.data)  # noqa: E731
    shp = np.array(shape, np.int64)
    off = np.empty(count + 1, np.int64)
    mx = ctypes.c_int64()
    nat.check(L.xhe_wire_begin(vp(ex), count, n2w, vp(shp), 1, int(framed), vp(off), ctypes.byref(mx), None, 0))
    out = nat.alloc_bytes(mx.value)
    optr = ctypes.c_void_p(ctypes.cast(out, ctypes.c_void_p).value)
    nat.check(L.xhe_wire_begin(vp(ex), count, n2w, vp(shp), 1, int(framed), vp(off), ctypes.byref(mx), optr, mx.value))
    bits = np.array([0 if not r.any() else 32 * int(np.nonzero(r)[0][-1]) + int(r[np.nonzero(r)[0][-1]]).bit_length()
                     for r in ct], np.int16)
    for k, lo in enumerate(range(0, count, 1234)):
        hi = min(count, lo + 1234)
        rows = np.ascontiguousarray(ct[lo:hi])
        if k % 2:  # the offsets from the rows' own words, or from device-style bit lengths
            nat.check(L.xhe_wire_layout_part_rows(vp(rows), vp(ex), lo, hi, count, n2w, vp(off)))
        else:
            b = np.ascontiguousarray(bits[lo:hi])
            nat.check(L.xhe_wire_layout_part(vp(b), vp(ex), lo, hi, count, n2w, vp(off)))
        nat.check(L.xhe_wire_rows(vp(rows), vp(ex), lo, hi, count, n2w, vp(off), int(framed), optr, mx.value))
    size = ctypes.c_int64()
    nat.check(L.xhe_wire_finish(count, vp(off), int(framed), optr, mx.value, ctypes.byref(size)))
    assert size.value <= mx.value
    box = [out]
    del out
    got = nat.shrink_bytes(box, size.value)
    if framed and len(wire.encode_words(ct, ex, shape)) >= compat.RAW_FRAME_MIN:
        assert got == want
    elif not framed:
        assert got == want
    assert compat.decompress(got) == wire.encode_words(ct, ex, shape) if framed else True


def test_shrink_bytes_in_place_and_shared():
    """nat.shrink_bytes cuts a payload it holds the only reference to in
    place (same prefix, no copy needed), and copies when something else still
    refers to the object (the other reference keeps its full bytes)."""
    b = nat.alloc_bytes(1 << 16)
    ctypes.memmove(ctypes.cast(b, ctypes.c_void_p).value, bytes(range(256)) * 256, 1 << 16)
    box = [b]
    del b
    got = nat.shrink_bytes(box, 1000)
    assert got == (bytes(range(256)) * 4)[:1000] and box == []
    big = nat.alloc_bytes(4096)
    ctypes.memset(ctypes.cast(big, ctypes.c_void_p).value, 7, 4096)
    keep = big
    box = [big]
    del big
    copies = nat.shrink_copies
    got2 = nat.shrink_bytes(box, 100)
    assert got2 == b"\x07" * 100 and len(keep) == 4096 and nat.shrink_copies == copies + 1
    with pytest.raises(ValueError):
        nat.shrink_bytes([bytes(10)], 20)


@pytest.mark.parametrize("count", [1, 2, 999, 1000, 1001, 2000, 5003])
def test_wire_begin_max_len_is_the_full_width_payload(count):
    """xhe_wire_begin's largest payload (closed form) is exactly the pickle of
    the same exponents with every value at n2w full words."""
    from xfl_amd.paillier import wire
    rng = np.random.default_rng(count)
    n2w = 128
    ex = rng.integers(-400, 700, count).astype(np.int32)
    full = np.full((count, n2w), 0xFFFFFFFF, np.uint32)
    want = len(wire.encode_words(full, ex, (count,)))
    L = nat.lib()
    vp = lambda a: ctypes.c_void_p(a.ctypes.data)  # noqa: E731
    off = np.empty(count + 1, np.int64)
    mx = ctypes.c_int64()
    shp = np.array([count], np.int64)
    nat.check(L.xhe_wire_begin(vp(ex), count, n2w, vp(shp), 1, 0, vp(off), ctypes.byref(mx), None, 0))
    assert mx.value == want
