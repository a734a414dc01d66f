"""CPU baseline worker for bench.py — TEST/BASELINE INFRASTRUCTURE ONLY.

Times the reference algorithm (DJN private-key CRT encryption,
paillier.py:189-209,273-287) restated in oracle/paillier_oracle.py with
pure-Python pow on this host; used as `cpu_baseline` (kind "port").
"""
import random
import time

from oracle import paillier_oracle as O

# fixed 2048/3072-bit DJN test keys are derived deterministically per worker
_KEYS = {}


def _key(bits):
    if bits not in _KEYS:
        from bench import make_key
        p, q, n, h = make_key(bits, seed=2024)
        _KEYS[bits] = O.derive_private(p, q, h)
    return _KEYS[bits]


def encrypt_for(arg):
    bits, seconds, wid = arg
    k = _key(bits)
    rng = random.Random(wid)
    bound = k["djn_exp_bound"]
    count = 0
    t0 = time.time()
    while time.time() - t0 < seconds:
        x = rng.gauss(0.0, 1.0)
        m, _ = O.encode_element(k, x, 7)
        O.encrypt_m(k, m, rng.randrange(1, bound))
        count += 1
    return count


# ---------------------------------------------------------------- GMP port
def _gmp_lib():
    import ctypes
    from oracle import build
    path = build.build()
    if path is None:
        return None
    L = ctypes.CDLL(path)
    if L.gmpb_load() != 0:
        return None
    return L


def _key_words(k, nw):
    import numpy as np

    def w(x, n):
        return np.frombuffer(int(x).to_bytes(4 * n, "little"), dtype="<u4").copy()

    return [w(k["n"], nw), w(k["n_square"], 2 * nw), w(k["p_square"], nw), w(k["q_square"], nw),
            w(k["q2_inverse_p2"], nw), w(k["h_pow_n_modp2"], nw), w(k["h_pow_n_modq2"], nw)]


def gmp_encrypt_one(k, m, a):
    """One DJN-CRT encryption through the GMP port (for checking it)."""
    import ctypes
    import numpy as np
    L = _gmp_lib()
    nw = (k["n"].bit_length() + 31) // 32
    arrs = _key_words(k, nw)
    aw = np.frombuffer(int(a).to_bytes(128, "little"), dtype="<u4").copy()
    out = np.zeros(2 * nw, dtype=np.uint32)
    args = [x.ctypes.data_as(ctypes.c_void_p) for x in arrs]
    rc = L.gmpb_encrypt_one(*args, ctypes.c_int(nw), ctypes.c_longlong(m), aw.ctypes.data_as(ctypes.c_void_p),
                            ctypes.c_int(32), out.ctypes.data_as(ctypes.c_void_p))
    assert rc == 0
    return int.from_bytes(out.tobytes(), "little")


def gmp_encrypt_batch(k, m_words, a_words, threads=8):
    """DJN-CRT private encryptions (1 + n m) h^a mod n^2 of encoded residues
    through the GMP port, many threads: the checker of the GPU parity tests at
    sizes the pure-Python oracle cannot finish in seconds. m_words [count][nw],
    a_words [count][aw] little-endian uint32; returns [count][2 nw] uint32."""
    import ctypes
    import numpy as np
    L = _gmp_lib()
    if L is None:
        raise RuntimeError("libgmp.so.10 not loadable: GMP checker unavailable")
    nw = (k["n"].bit_length() + 31) // 32
    m_words = np.ascontiguousarray(m_words, dtype=np.uint32)
    a_words = np.ascontiguousarray(a_words, dtype=np.uint32)
    count, aw = a_words.shape
    assert m_words.shape == (count, nw), (m_words.shape, count, nw)
    arrs = _key_words(k, nw)
    out = np.zeros((count, 2 * nw), dtype=np.uint32)
    vp = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    rc = L.gmpb_encrypt_batch(*[vp(x) for x in arrs], ctypes.c_int(nw), vp(m_words), vp(a_words), ctypes.c_int(aw),
                              ctypes.c_int64(count), ctypes.c_int(threads), vp(out))
    if rc != 0:
        raise RuntimeError(f"gmpb_encrypt_batch failed: {rc}")
    return out


def gmp_rate(bits, seconds, threads):
    """(encryptions, wall seconds) of the GMP port over `threads` threads, or None."""
    import ctypes
    L = _gmp_lib()
    if L is None:
        return None
    k = _key(bits)
    nw = bits // 32
    arrs = _key_words(k, nw)
    args = [x.ctypes.data_as(ctypes.c_void_p) for x in arrs]
    tot = ctypes.c_uint64()
    wall = ctypes.c_double()
    rc = L.gmpb_bench(*args, ctypes.c_int(nw), ctypes.c_double(seconds), ctypes.c_int(threads), ctypes.byref(tot),
                      ctypes.byref(wall))
    if rc != 0:
        return None
    return tot.value, wall.value
