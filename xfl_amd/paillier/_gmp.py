"""Key-generation arithmetic on the system GMP (ctypes), when it is present.

The reference generates keys with gmpy2 (`utils.py:79-89` getprimeover ->
`gmpy2.next_prime`, i.e. GMP's `mpz_nextprime`; `context.py:79-81` powmod ->
`mpz_powm`). This module calls the same two GMP routines through ctypes so a
4096/8192-bit key is generated in seconds rather than the minutes a pure-Python
Miller-Rabin takes; `next_prime` therefore returns exactly the prime gmpy2
would for the same starting point. Key generation is host-side and once per
`PaillierContext.generate` (per `fit()`), never on the per-element path.
Without libgmp the callers fall back to the pure-Python routines in utils.py.
"""
import ctypes
import ctypes.util


class _Mpz(ctypes.Structure):
    _fields_ = [("alloc", ctypes.c_int), ("size", ctypes.c_int), ("d", ctypes.c_void_p)]


def _load():
    for name in (ctypes.util.find_library("gmp"), "libgmp.so.10"):
        if not name:
            continue
        try:
            lib = ctypes.CDLL(name)
        except OSError:
            continue
        P = ctypes.POINTER(_Mpz)
        fns = {}
        for fn, res, args in (("__gmpz_init", None, [P]), ("__gmpz_clear", None, [P]),
                              ("__gmpz_set_str", ctypes.c_int, [P, ctypes.c_char_p, ctypes.c_int]),
                              ("__gmpz_get_str", ctypes.c_char_p, [ctypes.c_char_p, ctypes.c_int, P]),
                              ("__gmpz_sizeinbase", ctypes.c_size_t, [P, ctypes.c_int]),
                              ("__gmpz_nextprime", None, [P, P]),
                              ("__gmpz_powm", None, [P, P, P, P])):
            f = getattr(lib, fn)
            f.restype = res
            f.argtypes = args
            fns[fn[len("__gmpz_"):]] = f  # plain keys: no class-private name mangling
        return fns
    return None


_F = _load()


def available():
    return _F is not None


class _Z:
    """One mpz_t, set from / read back to a non-negative Python int via hex."""

    def __init__(self, v=0):
        self.z = _Mpz()
        _F["init"](ctypes.byref(self.z))
        if v:
            if _F["set_str"](ctypes.byref(self.z), format(v, "x").encode(), 16) != 0:
                raise ValueError("mpz_set_str failed")

    def value(self):
        n = _F["sizeinbase"](ctypes.byref(self.z), 16) + 2
        buf = ctypes.create_string_buffer(n)
        _F["get_str"](buf, 16, ctypes.byref(self.z))
        return int(buf.value, 16)

    def __del__(self):
        if _F is not None:
            _F["clear"](ctypes.byref(self.z))


def next_prime(x):
    """mpz_nextprime: the smallest probable prime > x (x >= 0)."""
    a, r = _Z(x), _Z()
    _F["nextprime"](ctypes.byref(r.z), ctypes.byref(a.z))
    return r.value()


def powmod(b, e, m):
    """mpz_powm for non-negative b, e and m > 0."""
    zb, ze, zm, r = _Z(b), _Z(e), _Z(m), _Z()
    _F["powm"](ctypes.byref(r.z), ctypes.byref(zb.z), ctypes.byref(ze.z), ctypes.byref(zm.z))
    return r.value()
