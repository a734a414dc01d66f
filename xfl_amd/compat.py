"""Wire compatibility with unmodified XFL peers (paillier.py:66-77,244-271).

* Pickles name `common.crypto.paillier.paillier.RawCiphertext`, as the
  reference's do; that module path is registered as an alias of
  xfl_amd.paillier.paillier unless a real XFL package is already importable.
* Reference pickles carry gmpy2 mpz values (`gmpy2.from_binary`); gmpy2 is not
  required here — `loads` maps that global to a decoder of gmpy2's binary
  format (b'\\x01' + sign byte + little-endian magnitude). Values we emit are
  Python ints, which the reference's gmpy2 arithmetic accepts unchanged.
* `compression=True` is zstd (the reference's `zstd.compress`): one standard
  frame with the content size in its header, which the reference's
  `zstd.decompress` reads. Payloads below 1 MiB are compressed by the system
  libzstd (level 3, through ctypes); larger ones - ciphertext arrays, of
  which level 3 keeps 98 % - are framed as raw blocks by the library's host
  threads (`xhe_zstd_raw_frame`), and such frames are read back by a
  parallel copy.
"""
import ctypes
import ctypes.util
import io
import threading
import pickle
import sys
import types

_REF_MOD = "common.crypto.paillier.paillier"


def _register_alias():
    from .paillier import paillier as mod
    if _REF_MOD in sys.modules:
        return
    try:  # a real XFL install wins
        __import__(_REF_MOD)
        return
    except Exception:
        pass
    for name in ("common", "common.crypto", "common.crypto.paillier"):
        if name not in sys.modules:
            m = types.ModuleType(name)
            m.__path__ = []
            sys.modules[name] = m
    sys.modules[_REF_MOD] = mod


def gmpy2_from_binary(b):
    """Decode gmpy2.to_binary(mpz) (type byte 0x01, sign 0x01/0x02)."""
    b = bytes(b)
    if len(b) < 2 or b[0] != 0x01:
        raise pickle.UnpicklingError("unsupported gmpy2 binary object")
    mag = int.from_bytes(b[2:], "little")
    return -mag if b[1] == 0x02 else mag


# Globals a ciphertext / context / RawCiphertext payload may name
# (paillier.py:244-271, context.py:152-168): numpy's ndarray reduce (numpy 1.x
# and 2.x module paths), numpy scalars (an exponent can be an np.int32 taken
# from np.frexp), protocol-0/1 object reconstruction and plain builtins.
# Anything else raises instead of importing: peer bytes are untrusted.
_ALLOWED = {
    ("numpy.core.multiarray", "_reconstruct"), ("numpy._core.multiarray", "_reconstruct"),
    ("numpy.core.multiarray", "scalar"), ("numpy._core.multiarray", "scalar"),
    ("numpy", "ndarray"), ("numpy", "dtype"),
    ("copyreg", "_reconstructor"), ("copy_reg", "_reconstructor"),
    ("builtins", "object"), ("__builtin__", "object"),
    ("builtins", "int"), ("builtins", "float"), ("builtins", "tuple"), ("builtins", "list"),
    ("builtins", "dict"), ("builtins", "bytes"), ("builtins", "str"), ("builtins", "complex"),
    ("_codecs", "encode"),  # protocol < 3 pickles of bytes
}


class _Unpickler(pickle.Unpickler):
    def find_class(self, module, name):
        if module == "gmpy2" and name == "from_binary":
            return gmpy2_from_binary
        if module == _REF_MOD and name == "RawCiphertext":
            from .paillier.paillier import RawCiphertext
            return RawCiphertext
        if (module, name) in _ALLOWED:
            return super().find_class(module, name)
        raise pickle.UnpicklingError(f"global {module}.{name} is not allowed in a Paillier payload")


def dumps(obj) -> bytes:
    _register_alias()
    return pickle.dumps(obj)


def loads(data: bytes):
    _register_alias()
    return _Unpickler(io.BytesIO(data)).load()


# ------------------------------------------------------------------ zstd
_zstd = None


def _lib():
    global _zstd
    if _zstd is None:
        path = ctypes.util.find_library("zstd") or "libzstd.so.1"
        L = ctypes.CDLL(path)
        L.ZSTD_compressBound.restype = ctypes.c_size_t
        L.ZSTD_compressBound.argtypes = [ctypes.c_size_t]
        L.ZSTD_compress.restype = ctypes.c_size_t
        L.ZSTD_compress.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        L.ZSTD_decompress.restype = ctypes.c_size_t
        L.ZSTD_decompress.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t]
        L.ZSTD_getFrameContentSize.restype = ctypes.c_ulonglong
        L.ZSTD_getFrameContentSize.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
        L.ZSTD_isError.restype = ctypes.c_uint
        L.ZSTD_isError.argtypes = [ctypes.c_size_t]
        _zstd = L
    return _zstd


_scratch = threading.local()


def _dst(cap):
    """per-thread output buffer, kept between calls (already paged in)"""
    import numpy as np
    buf = getattr(_scratch, "buf", None)
    if buf is None or buf.shape[0] < cap:
        buf = _scratch.buf = np.empty(cap, dtype=np.uint8)
    return buf


RAW_FRAME_MIN = 1 << 20  # payloads from this size up are framed as raw blocks


def compress(data: bytes, level: int = 3) -> bytes:
    """zstd frame of data (the reference's zstd.compress, paillier.py:244-258):
    one frame, content size in the header. Payloads of RAW_FRAME_MIN bytes
    and more - ciphertext arrays, 98 % incompressible at level 3 - become one
    frame of raw blocks written by the library's host threads
    (xhe_zstd_raw_frame); smaller ones are compressed by libzstd."""
    if len(data) >= RAW_FRAME_MIN:
        from . import _native as nat
        L = nat.lib()
        size = L.xhe_zstd_raw_frame_size(len(data))
        out = nat.alloc_bytes(size)  # written in place (every byte); nothing else references it yet
        ptr = ctypes.cast(out, ctypes.c_void_p)
        n = ctypes.c_int64()
        nat.check(L.xhe_zstd_raw_frame(data, len(data), ptr, size, ctypes.byref(n)), "zstd frame")
        return out
    L = _lib()
    cap = L.ZSTD_compressBound(len(data))
    dst = _dst(cap)
    n = L.ZSTD_compress(dst.ctypes.data, cap, data, len(data), level)
    if L.ZSTD_isError(n):
        raise RuntimeError("zstd compression failed")
    return dst[:n].tobytes()


def _raw_extract(data):
    """content of a raw-block frame (parallel copy), or None for any other frame"""
    from . import _native as nat
    try:
        L = nat.lib()
    except Exception:
        return None
    n = ctypes.c_int64()
    if L.xhe_zstd_raw_extract(data, len(data), None, 0, ctypes.byref(n)) != nat.XHE_EOVERFLOW or n.value < 2:
        return None
    out = nat.alloc_bytes(n.value)  # every byte written by the extract
    ptr = ctypes.cast(out, ctypes.c_void_p)
    nat.check(L.xhe_zstd_raw_extract(data, len(data), ptr, n.value, ctypes.byref(n)), "zstd extract")
    return out


def decompress(data: bytes) -> bytes:
    if len(data) >= RAW_FRAME_MIN:
        out = _raw_extract(data)
        if out is not None:
            return out
    L = _lib()
    size = L.ZSTD_getFrameContentSize(data, len(data))
    if size >= (1 << 63):  # unknown / error
        raise RuntimeError("zstd frame without content size")
    if size < 2:  # bytes(0) / bytes(1) are shared singletons: never write into them
        dst = ctypes.create_string_buffer(max(int(size), 1))
        n = L.ZSTD_decompress(dst, int(size), data, len(data))
        if L.ZSTD_isError(n):
            raise RuntimeError("zstd decompression failed")
        return ctypes.string_at(dst, n)
    from . import _native as nat
    out = nat.alloc_bytes(int(size))  # written in place: the frame fills it exactly
    n = L.ZSTD_decompress(ctypes.cast(out, ctypes.c_void_p), int(size), data, len(data))
    if L.ZSTD_isError(n) or n != size:
        raise RuntimeError("zstd decompression failed")
    return out
