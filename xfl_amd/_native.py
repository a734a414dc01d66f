"""ctypes binding of the xhe C ABI (include/xhe.h) built from xfl_amd/csrc.

The shared library is built in-tree (xfl_amd/lib/libxhe.so) by
`__graft_entry__.build()` / `python -m xfl_amd.build`. There is no CPU
fallback: if the library or a GPU is missing, every entry point raises.
"""
import ctypes
import mmap
import os
import sys
import threading
import weakref

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("XHE_LIB", os.path.join(_HERE, "lib", "libxhe.so"))  # XHE_LIB: A/B builds

XHE_OK = 0
XHE_EINVAL = -1
XHE_EOVERFLOW = -2
XHE_EHIP = -3
XHE_ENOINV = -4
XHE_ENOTSUP = -5

_lib = None
_lock = threading.Lock()

_u32p = ctypes.POINTER(ctypes.c_uint32)
_i32p = ctypes.POINTER(ctypes.c_int32)
_vp = ctypes.c_void_p

# name -> (restype, argtypes); every symbol declared in include/xhe.h
SIGNATURES = {
    "xhe_key_create": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, _u32p, _u32p, _u32p, _u32p, ctypes.c_int,
                                      ctypes.POINTER(_vp)]),
    "xhe_key_destroy": (None, [_vp]),
    "xhe_key_info": (ctypes.c_int, [_vp] + [ctypes.POINTER(ctypes.c_int)] * 6),
    "xhe_encode_f64": (ctypes.c_int, [_vp, _vp, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                      _vp, _vp, _vp, _vp]),
    "xhe_rand": (ctypes.c_int, [_vp, ctypes.c_char_p, ctypes.c_uint64, ctypes.c_int64, _vp, _vp, _vp]),
    "xhe_encrypt": (ctypes.c_int, [_vp, _vp, _vp, ctypes.c_int64, _vp, _vp]),
    "xhe_decrypt": (ctypes.c_int, [_vp, _vp, ctypes.c_int64, _vp, _vp]),
    "xhe_decode": (ctypes.c_int, [_vp, _vp, _vp, ctypes.c_int64, _vp, _vp, _vp, _vp]),
    "xhe_mulmod": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, ctypes.c_int64, ctypes.c_int, _vp, _vp, _vp]),
    "xhe_powmod": (ctypes.c_int, [_vp, _vp, _vp, ctypes.c_int, ctypes.c_int, ctypes.c_int64, _vp, _vp]),
    "xhe_invert": (ctypes.c_int, [_vp, _vp, ctypes.c_int64, _vp, _vp]),
    "xhe_mulmod_host": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, ctypes.c_int64, ctypes.c_int, _vp, _vp]),
    "xhe_powmod_host": (ctypes.c_int, [_vp, _vp, _vp, ctypes.c_int, ctypes.c_int, ctypes.c_int64, ctypes.c_int,
                                       _vp]),
    "xhe_segprod": (ctypes.c_int, [_vp, _vp, _vp, ctypes.c_int, ctypes.c_int64, _vp, ctypes.c_int64, _vp, _vp]),
    "xhe_segprod_host": (ctypes.c_int, [_vp, _vp, _vp, ctypes.c_int, ctypes.c_int64, _vp, ctypes.c_int64, _vp]),
    "xhe_gather_rows": (ctypes.c_int, [_vp, _vp, ctypes.c_int64, ctypes.c_int, _vp, _vp]),
    "xhe_scatter_rows": (ctypes.c_int, [_vp, _vp, ctypes.c_int64, ctypes.c_int, _vp, _vp]),
    "xhe_multiexp": (ctypes.c_int, [_vp, _vp, ctypes.c_int64, _vp, _vp, ctypes.c_int, ctypes.c_int, ctypes.c_int64,
                                    ctypes.c_int64, ctypes.c_int, _vp, _vp]),
    "xhe_multiexp_host": (ctypes.c_int, [_vp, _vp, ctypes.c_int64, _vp, _vp, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_int64, ctypes.c_int64, ctypes.c_int, _vp]),
    "xhe_encrypt_host": (ctypes.c_int, [_vp, _vp, _vp, ctypes.c_int64, _vp]),
    "xhe_decrypt_host": (ctypes.c_int, [_vp, _vp, ctypes.c_int64, _vp]),
    "xhe_encrypt_f64_host": (ctypes.c_int, [_vp, _vp, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                            ctypes.c_int, ctypes.c_char_p, ctypes.c_uint64, _vp, _vp, _vp]),
    "xhe_encrypt_words_host": (ctypes.c_int, [_vp, _vp, ctypes.c_int64, ctypes.c_int, ctypes.c_char_p,
                                              ctypes.c_uint64, _vp]),
    "xhe_decrypt_decode_host": (ctypes.c_int, [_vp, _vp, _vp, ctypes.c_int64, _vp, _vp, _vp, _vp]),
    "xhe_wire_encode": (ctypes.c_int, [_vp, _vp, ctypes.c_int64, ctypes.c_int, _vp, ctypes.c_int, _vp,
                                       ctypes.c_int64, ctypes.POINTER(ctypes.c_int64)]),
    "xhe_wire_encode_frame": (ctypes.c_int, [_vp, _vp, ctypes.c_int64, ctypes.c_int, _vp, ctypes.c_int, ctypes.c_int,
                                             _vp, ctypes.c_int64, ctypes.POINTER(ctypes.c_int64)]),
    "xhe_wire_layout": (ctypes.c_int, [_vp, _vp, ctypes.c_int64, ctypes.c_int, _vp, ctypes.c_int, ctypes.c_int, _vp,
                                       _vp, ctypes.c_int64, ctypes.POINTER(ctypes.c_int64)]),
    "xhe_wire_rows": (ctypes.c_int, [_vp, _vp, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int, _vp,
                                     ctypes.c_int, _vp, ctypes.c_int64]),
    "xhe_wire_begin": (ctypes.c_int, [_vp, ctypes.c_int64, ctypes.c_int, _vp, ctypes.c_int, ctypes.c_int, _vp,
                                      ctypes.POINTER(ctypes.c_int64), _vp, ctypes.c_int64]),
    "xhe_wire_layout_part": (ctypes.c_int, [_vp, _vp, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int,
                                            _vp]),
    "xhe_wire_layout_part_rows": (ctypes.c_int, [_vp, _vp, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                                                 ctypes.c_int, _vp]),
    "xhe_wire_finish": (ctypes.c_int, [ctypes.c_int64, _vp, ctypes.c_int, _vp, ctypes.c_int64,
                                       ctypes.POINTER(ctypes.c_int64)]),
    "xhe_row_bits": (ctypes.c_int, [_vp, ctypes.c_int64, ctypes.c_int, _vp, _vp]),
    "xhe_rns_constants": (ctypes.c_int, [_vp, ctypes.c_int, _vp, _vp]),
    "xhe_wire_decode": (ctypes.c_int, [_vp, ctypes.c_int64, ctypes.c_int, _vp, _vp, ctypes.c_int64,
                                       ctypes.POINTER(ctypes.c_int64), _vp, ctypes.POINTER(ctypes.c_int)]),
    "xhe_host_prefault": (ctypes.c_int, [_vp, ctypes.c_int64]),
    "xhe_zstd_raw_frame_size": (ctypes.c_int64, [ctypes.c_int64]),
    "xhe_zstd_raw_frame": (ctypes.c_int, [_vp, ctypes.c_int64, _vp, ctypes.c_int64, ctypes.POINTER(ctypes.c_int64)]),
    "xhe_zstd_raw_extract": (ctypes.c_int, [_vp, ctypes.c_int64, _vp, ctypes.c_int64,
                                            ctypes.POINTER(ctypes.c_int64)]),
    "xhe_profile": (ctypes.c_int, [ctypes.c_int]),
    "xhe_profile_read": (ctypes.c_int, [ctypes.c_char_p, ctypes.POINTER(ctypes.c_double),
                                        ctypes.POINTER(ctypes.c_int64)]),
    "xhe_device_count": (ctypes.c_int, []),
    "xhe_synchronize": (ctypes.c_int, [_vp]),
    "xhe_last_error": (ctypes.c_char_p, []),
    "xhe_version": (ctypes.c_char_p, []),
}


class XheError(RuntimeError):
    pass


def lib():
    """Load libxhe.so once; raise loudly if it is missing (no CPU fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise XheError(f"xfl_amd native library not built: {LIB_PATH} missing "
                               "(run __graft_entry__.build())")
            # One HIP runtime per process: PyTorch-ROCm bundles its own
            # libamdhip64. Loading torch first makes libxhe bind to that copy;
            # the other order leaves torch.cuda with "No HIP GPUs" later in
            # the same process (XFL's operators import torch anyway).
            try:
                import torch  # noqa: F401
            except ImportError:
                pass
            L = ctypes.CDLL(LIB_PATH)
            for name, (res, args) in SIGNATURES.items():
                try:
                    fn = getattr(L, name)
                except AttributeError:
                    if "XHE_LIB" in os.environ:  # an older A/B build: bind what it has
                        continue
                    raise
                fn.restype = res
                fn.argtypes = args
            _lib = L
    return _lib


_ndev = None


def visible_devices():
    """GPUs visible to this process (cached)."""
    global _ndev
    if _ndev is None:
        _ndev = max(1, int(lib().xhe_device_count()))
    return _ndev


def check(rc, what=""):
    if rc == XHE_OK:
        return
    msg = lib().xhe_last_error().decode(errors="replace")
    if rc == XHE_EOVERFLOW:
        raise OverflowError(msg)
    if rc == XHE_ENOINV:
        raise ZeroDivisionError(msg)
    if rc == XHE_EINVAL:
        raise ValueError(f"{what}: {msg}")
    raise XheError(f"{what} failed ({rc}): {msg}")


# ------------------------------------------------------------ host buffers
_libc = None
_HUGE = 2 << 20
_MADV_HUGEPAGE = 14


def advise_huge(addr, nbytes):
    """madvise(MADV_HUGEPAGE) on the 2 MiB-aligned interior of a fresh buffer:
    the ciphertext payloads are hundreds of MB, and first-touch faults at 4 KiB
    cost more than writing them (transparent hugepages are 'madvise' mode on
    these hosts). Best effort: ignored where unsupported."""
    global _libc
    if nbytes < (32 << 20):
        return
    try:
        if _libc is None:
            _libc = ctypes.CDLL(None)
            _libc.madvise.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        lo = (addr + _HUGE - 1) & ~(_HUGE - 1)
        hi = (addr + nbytes) & ~(_HUGE - 1)
        if hi > lo:
            _libc.madvise(lo, hi - lo, _MADV_HUGEPAGE)
    except (OSError, AttributeError):
        pass


_M_TRIM_THRESHOLD, _M_MMAP_MAX, _M_MMAP_MAX_DEFAULT = -1, -4, 65536
_heap_lock = threading.Lock()
_heap_ready = False
HEAP_PAYLOAD_MAX = (1 << 31) - 1  # payloads up to this size come from the heap (below); mallopt takes an int


def _pybytes(n):
    f = ctypes.pythonapi.PyBytes_FromStringAndSize
    f.restype = ctypes.py_object
    f.argtypes = [ctypes.c_void_p, ctypes.c_ssize_t]
    return f(None, n)


shrink_copies = 0  # shrink_bytes calls that had to copy (tests check the pipeline never does)


def shrink_bytes(box, n):
    """box: a one-element list holding the only reference to a bytes object
    (from alloc_bytes); returns that object cut to its first n bytes in place
    (_PyBytes_Resize: a realloc that keeps the block, no copy) - the
    serialize pipeline allocates the largest payload its elements could need
    before their sizes are known. Falls back to a copy when anything else
    still refers to the object."""
    b = box.pop()
    n = int(n)
    if n == len(b):
        return b
    if not 2 <= n < len(b):
        raise ValueError("shrink_bytes: n must be in [2, len)")
    if sys.getrefcount(b) != 2:  # b + getrefcount's argument
        global shrink_copies
        shrink_copies += 1
        return b[:n]
    api = ctypes.pythonapi
    api.Py_IncRef.argtypes = [ctypes.c_void_p]
    api.Py_DecRef.argtypes = [ctypes.c_void_p]
    api.Py_NewRef.argtypes = [ctypes.c_void_p]
    api.Py_NewRef.restype = ctypes.py_object
    api._PyBytes_Resize.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_ssize_t]
    api._PyBytes_Resize.restype = ctypes.c_int
    slot = ctypes.c_void_p(id(b))
    api.Py_IncRef(slot.value)  # the slot's own reference, the only one after del
    del b
    if api._PyBytes_Resize(ctypes.byref(slot), n) != 0:  # (the object is gone then)
        raise MemoryError("shrink_bytes: _PyBytes_Resize failed")
    out = api.Py_NewRef(slot.value)
    api.Py_DecRef(slot.value)
    return out


def alloc_bytes(n):
    """An UNINITIALISED bytes object of n bytes for the library to fill
    completely (the serialize payloads: Paillier.serialize returns bytes,
    paillier.py:244-258). Payloads of 32 MiB up to HEAP_PAYLOAD_MAX are taken
    from glibc's main heap rather than a fresh mapping: on the GPU box a
    545 MB mapping cost its first-touch faults and ~30 ms more when it was
    unmapped (the kernel zeroes freed pages), once per payload; a heap block
    freed by the caller stays in the heap's free list (trimming raised to
    2 GiB) and the next payload of a training loop lands in the same, already
    mapped pages. Main thread only (another thread's arena cannot grow that
    far without mmap); $XHE_HEAP_PAYLOADS=0 turns it off."""
    global _heap_ready
    n = int(n)
    if n < 2:
        raise ValueError("alloc_bytes: bytes objects below 2 bytes are shared singletons")
    if n < (32 << 20) or n > HEAP_PAYLOAD_MAX or os.environ.get("XHE_HEAP_PAYLOADS", "1").strip() == "0" or \
            threading.current_thread() is not threading.main_thread():
        b = _pybytes(n)
        advise_huge(ctypes.cast(b, ctypes.c_void_p).value, n)
        return b
    global _libc
    with _heap_lock:
        try:
            if _libc is None:
                _libc = ctypes.CDLL(None)
                _libc.madvise.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
            _libc.mallopt.argtypes = [ctypes.c_int, ctypes.c_int]
            if not _heap_ready:
                _libc.mallopt(_M_TRIM_THRESHOLD, HEAP_PAYLOAD_MAX)  # freed payload blocks stay in the heap
                _heap_ready = True
            _libc.mallopt(_M_MMAP_MAX, 0)
            try:
                return _pybytes(n)
            finally:
                _libc.mallopt(_M_MMAP_MAX, _M_MMAP_MAX_DEFAULT)
        except (MemoryError, OSError, AttributeError):
            pass
    b = _pybytes(n)
    advise_huge(ctypes.cast(b, ctypes.c_void_p).value, n)
    return b


class _HostBlock:
    """Owner (the numpy base) of a recycled host allocation."""
    __slots__ = ("__array_interface__", "mem", "__weakref__")


_pool_lock = threading.Lock()
_pool_free = {}       # nbytes -> [mmap]
_pool_bytes = 0
POOL_MAX_BYTES = 8 << 30   # freed result buffers kept for reuse, at most
POOL_PER_SIZE = 4


def _pool_release(mem, nbytes):
    global _pool_bytes
    with _pool_lock:
        lst = _pool_free.setdefault(nbytes, [])
        if _pool_bytes + nbytes <= POOL_MAX_BYTES and len(lst) < POOL_PER_SIZE:
            lst.append(mem)
            _pool_bytes += nbytes
            return
    # dropped: unmapped when the last reference goes


def _pool_take(nbytes):
    global _pool_bytes
    with _pool_lock:
        lst = _pool_free.get(nbytes)
        if lst:
            _pool_bytes -= nbytes
            return lst.pop()
    return None


def empty(shape, dtype):
    """np.empty for the large host buffers the library writes results into
    (ciphertext arrays of hundreds of MB). They come from a small cache of
    anonymous mappings: when every array on a buffer has been released its
    pages go back to the cache (up to POOL_MAX_BYTES), so a training loop's
    next result of the same size lands in pages that are already faulted in
    instead of paying the kernel's first-touch zero-fill again. Fresh mappings
    are hugepage-advised and pre-faulted by the library's host threads."""
    dt = np.dtype(dtype)
    shape = tuple(int(d) for d in (shape if isinstance(shape, (tuple, list)) else (shape,)))
    nbytes = int(np.prod(shape, dtype=np.int64)) * dt.itemsize
    if nbytes < (32 << 20):
        return np.empty(shape, dtype=dt)
    mem = _pool_take(nbytes)
    fresh = mem is None
    if fresh:
        mem = mmap.mmap(-1, nbytes)
    addr = ctypes.addressof(ctypes.c_char.from_buffer(mem))
    if fresh:
        advise_huge(addr, nbytes)
        lib().xhe_host_prefault(ctypes.c_void_p(addr), ctypes.c_int64(nbytes))
    owner = _HostBlock()
    owner.mem = mem
    owner.__array_interface__ = {"data": (addr, False), "shape": shape, "typestr": dt.str, "version": 3}
    a = np.asarray(owner)
    weakref.finalize(owner, _pool_release, mem, nbytes)
    return a


# ------------------------------------------------------------ int <-> words
def int_to_words(x, nw):
    return np.frombuffer(int(x).to_bytes(4 * nw, "little"), dtype="<u4").copy()


def ints_to_words(xs, nw):
    nb = 4 * nw
    tb = int.to_bytes
    buf = bytearray().join([tb(int(x), nb, "little") for x in xs])
    return np.frombuffer(buf, dtype="<u4").reshape(len(xs), nw)


def words_to_ints(w):
    w = np.ascontiguousarray(w, dtype="<u4")
    if w.ndim == 1:
        return int.from_bytes(w.tobytes(), "little")
    nb = w.shape[1] * 4
    mv = memoryview(w).cast("B")  # no copy
    fb = int.from_bytes
    return [fb(mv[i * nb:(i + 1) * nb], "little") for i in range(w.shape[0])]


def ptr(a):
    return a.ctypes.data_as(_u32p)


TABLE_ROW_WORDS = {2048: 64, 3072: 96, 4096: 128, 8192: 256}  # packed rows: xhe.hip Shape<K>::RW = K/32


XHE_WIN_SPLIT = 0x100  # include/xhe.h: floor(rand_bits/w) windows, the first rand_bits mod w of them w+1 bits


def win_layout(rand_bits, win_bits):
    """(windows, wide windows) of a fixed-base table (xhe.hip win_layout):
    ceil(rand_bits/w) windows of w bits, or with XHE_WIN_SPLIT floor(rand_bits/w)
    windows of which the first rand_bits mod w are w+1 bits wide."""
    w = win_bits & 0xFF
    if win_bits & XHE_WIN_SPLIT and rand_bits % w and rand_bits % w <= rand_bits // w:
        return rand_bits // w, rand_bits % w
    return -(-rand_bits // w), 0


def win_spec(win_bits):
    """'23' / '23s' (split) - the text form of a window choice."""
    return f"{win_bits & 0xFF}{'s' if win_bits & XHE_WIN_SPLIT else ''}"


def parse_win(spec):
    """Inverse of win_spec; also accepts plain ints."""
    spec = str(spec).strip()
    return int(spec[:-1]) | XHE_WIN_SPLIT if spec.endswith("s") else int(spec)


def table_bytes(key_bits, win_bits):
    """Device bytes of a DJN private key's two fixed-base tables: per prime
    (windows + wide windows) x 2^w packed rows of K/32 words (rand_bits = K/2)."""
    if not win_bits:
        return 0
    nwin, nhi = win_layout(key_bits // 2, win_bits)
    return 2 * (nwin + nhi) * (1 << (win_bits & 0xFF)) * TABLE_ROW_WORDS[key_bits] * 4


def device_free_bytes(device=0):
    """Free HBM on `device` (None when it cannot be queried)."""
    try:
        import torch
        return int(torch.cuda.mem_get_info(device)[0])
    except Exception:
        return None


class DeviceKey:
    """Owns one xhe_key handle (device-resident key constants and tables)."""

    def __init__(self, key_bits, n, p=None, q=None, h_pow_n=None, device=0, win_bits=0):
        L = lib()
        self.key_bits = key_bits
        self.nw = key_bits // 32
        self.n2w = 2 * self.nw
        nw_ = int_to_words(n, self.nw)
        pw = int_to_words(p, self.nw // 2) if p is not None else None
        qw = int_to_words(q, self.nw // 2) if q is not None else None
        hw = int_to_words(h_pow_n, self.n2w) if h_pow_n else None
        h = _vp()
        rc = L.xhe_key_create(device, key_bits, ptr(nw_), ptr(pw) if pw is not None else None,
                              ptr(qw) if qw is not None else None, ptr(hw) if hw is not None else None,
                              win_bits, ctypes.byref(h))
        check(rc, "xhe_key_create")
        self.handle = h
        vals = [ctypes.c_int() for _ in range(6)]
        check(L.xhe_key_info(h, *[ctypes.byref(v) for v in vals]), "xhe_key_info")
        _, _, _, self.rand_words, self.rand_bits, flags = [v.value for v in vals]
        self.private = bool(flags & 1)
        self.djn = bool(flags & 2)
        self.device = device
        wb = (win_bits or parse_win(os.environ.get("XHE_WIN_BITS", "0") or 16)) if self.private and self.djn else 0
        self.win_bits = wb & 0xFF  # the window w
        self.win_split = bool(wb & XHE_WIN_SPLIT)

    def __del__(self):
        h = getattr(self, "handle", None)
        if h and _lib is not None:
            _lib.xhe_key_destroy(h)
            self.handle = None

    # host-buffer paths (used by the drop-in API)
    def encrypt_words(self, m_words, rand_words):
        m_words = np.ascontiguousarray(m_words, dtype=np.uint32)
        count = m_words.shape[0]
        out = np.empty((count, self.n2w), dtype=np.uint32)
        if count == 0:
            return out
        r = None if rand_words is None else np.ascontiguousarray(rand_words, dtype=np.uint32)
        check(lib().xhe_encrypt_host(self.handle, ptr(m_words), ptr(r) if r is not None else None, count,
                                     ptr(out)), "xhe_encrypt")
        return out

    def decrypt_words(self, c_words):
        c_words = np.ascontiguousarray(c_words, dtype=np.uint32)
        count = c_words.shape[0]
        out = np.empty((count, self.nw), dtype=np.uint32)
        if count == 0:
            return out
        check(lib().xhe_decrypt_host(self.handle, ptr(c_words), count, ptr(out)), "xhe_decrypt")
        return out
