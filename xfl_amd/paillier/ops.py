"""Batched device operations behind the drop-in API.

Every function takes/returns Python ints (the reference's mpz role) and runs
the arithmetic on the GPU through the xhe C ABI (include/xhe.h). There is no
CPU arithmetic path: a missing library or GPU raises from xfl_amd._native.
"""
import ctypes
import itertools
import os

import numpy as np

from .. import _native as nat

_nonce = itertools.count(1)


def _seed():
    return os.urandom(32), next(_nonce)


def _u32(a):
    return np.ascontiguousarray(a, dtype=np.uint32)


def _i32(a):
    return np.ascontiguousarray(a, dtype=np.int32)


def _vp(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None else None


def encrypt_floats(ctx, xs, precision, max_exponent, obfuscation):
    """encode (device) + encrypt for float64 values -> (raw ints, exponents, status)."""
    dk = ctx.device_key()
    x = np.ascontiguousarray(xs, dtype=np.float64)
    n = x.shape[0]
    ct = np.empty((n, dk.n2w), dtype=np.uint32)
    ex = np.empty(n, dtype=np.int32)
    st = np.empty(n, dtype=np.int32)
    if n == 0:
        return [], ex, st
    seed, nonce = _seed()
    prec = -1 if precision is None else int(precision)
    has_max = max_exponent is not None
    nat.check(nat.lib().xhe_encrypt_f64_host(dk.handle, _vp(x), n, prec, int(has_max),
                                             int(max_exponent) if has_max else 0, int(bool(obfuscation)),
                                             seed, nonce, _vp(ct), _vp(ex), _vp(st)), "encrypt")
    return nat.words_to_ints(ct), ex, st


def encrypt_encoded(ctx, ms, obfuscation):
    """encrypt already-encoded integers m (0 <= m < n)."""
    dk = ctx.device_key()
    n = len(ms)
    if n == 0:
        return []
    mw = nat.ints_to_words(ms, dk.nw)
    ct = np.empty((n, dk.n2w), dtype=np.uint32)
    seed, nonce = _seed()
    nat.check(nat.lib().xhe_encrypt_words_host(dk.handle, _vp(mw), n, int(bool(obfuscation)), seed, nonce,
                                               _vp(ct)), "encrypt")
    return nat.words_to_ints(ct)


def decrypt_ints(ctx, raws):
    """decrypt -> encoded integers m (paillier.py:347-365)."""
    dk = ctx.device_key()
    if len(raws) == 0:
        return []
    return nat.words_to_ints(dk.decrypt_words(nat.ints_to_words(raws, dk.n2w)))


def decrypt_float32(ctx, raws, exps):
    """decrypt + decode + float32 on the device -> (f64, f32, status)."""
    dk = ctx.device_key()
    n = len(raws)
    cw = nat.ints_to_words(raws, dk.n2w)
    e = _i32(exps)
    f64 = np.empty(n, dtype=np.float64)
    f32 = np.empty(n, dtype=np.float32)
    st = np.empty(n, dtype=np.int32)
    if n:
        nat.check(nat.lib().xhe_decrypt_decode_host(dk.handle, _vp(cw), _vp(e), n, _vp(f64), _vp(f32), _vp(st),
                                                    None), "decrypt")
    return f64, f32, st


def add(ctx, ra, ea, rb, eb):
    """ciphertext + ciphertext with exponent alignment -> (raws, exps)."""
    dk = ctx.device_key()
    n = len(ra)
    if n == 0:
        return [], np.empty(0, dtype=np.int32)
    aw = nat.ints_to_words(ra, dk.n2w)
    bw = nat.ints_to_words(rb, dk.n2w)
    ea = _i32(ea)
    eb = _i32(eb)
    dmax = int(np.max(np.abs(ea.astype(np.int64) - eb.astype(np.int64)))) if n else 0
    out = np.empty((n, dk.n2w), dtype=np.uint32)
    eo = np.empty(n, dtype=np.int32)
    nat.check(nat.lib().xhe_mulmod_host(dk.handle, _vp(aw), _vp(ea), _vp(bw), _vp(eb), n, dmax, _vp(out),
                                        _vp(eo)), "add")
    return nat.words_to_ints(out), eo


def powmod(ctx, raws, ks, invert_first=False):
    """c^k (or (c^-1)^k) mod n^2 for per-element k >= 0."""
    dk = ctx.device_key()
    n = len(raws)
    if n == 0:
        return []
    kbits = max(int(k).bit_length() for k in ks)
    kw = max(1, (kbits + 31) // 32)
    cw = nat.ints_to_words(raws, dk.n2w)
    kwds = nat.ints_to_words(ks, kw)
    out = np.empty((n, dk.n2w), dtype=np.uint32)
    nat.check(nat.lib().xhe_powmod_host(dk.handle, _vp(cw), _vp(kwds), kw, kbits, n, int(bool(invert_first)),
                                        _vp(out)), "powmod")
    return nat.words_to_ints(out)


def raw_mul(ctx, raws, ks):
    """PaillierCiphertext._raw_mul for 0 <= k < n (paillier.py:156-187):
    inv(c)^(n-k) when k >= min_value_for_negative, else c^k."""
    n = len(raws)
    out = [None] * n
    thr = ctx.min_value_for_negative
    pos = [i for i in range(n) if ks[i] < thr]
    neg = [i for i in range(n) if ks[i] >= thr]
    if pos:
        r = powmod(ctx, [raws[i] for i in pos], [ks[i] for i in pos])
        for i, v in zip(pos, r):
            out[i] = v
    if neg:
        r = powmod(ctx, [raws[i] for i in neg], [ctx.n - ks[i] for i in neg], invert_first=True)
        for i, v in zip(neg, r):
            out[i] = v
    return out


def obfuscate(ctx, raws):
    """PaillierCiphertext.obfuscate: c * X with X a fresh obfuscator (= encryption of 0)."""
    n = len(raws)
    if n == 0:
        return []
    xs = encrypt_encoded(ctx, [0] * n, True)
    z = np.zeros(n, dtype=np.int32)
    r, _ = add(ctx, raws, z, xs, z)
    return r


def multiexp(ctx, bases, idx, ks, win_bits=0):
    """out[j] = prod_t bases[idx[j][t]]^ks[j][t] mod n^2 (ks >= 0): one
    xhe_multiexp call (Straus windows, per-base tables shared by all j)."""
    dk = ctx.device_key()
    ncols = len(idx)
    nterms = len(idx[0]) if ncols else 0
    if ncols == 0 or nterms == 0 or not bases:
        raise ValueError("multiexp: empty problem")
    flat_k = [int(k) for row in ks for k in row]
    kbits = max(1, max(k.bit_length() for k in flat_k))
    kw = (kbits + 31) // 32
    bw = nat.ints_to_words(bases, dk.n2w)
    iw = np.ascontiguousarray(idx, dtype=np.int32).reshape(ncols, nterms)
    kwds = nat.ints_to_words(flat_k, kw)
    out = np.empty((ncols, dk.n2w), dtype=np.uint32)
    nat.check(nat.lib().xhe_multiexp_host(dk.handle, _vp(bw), len(bases), _vp(iw), _vp(kwds), kw, kbits, ncols,
                                          nterms, int(win_bits), _vp(out)), "multiexp")
    return nat.words_to_ints(out)


def segment_sums(ctx, raws, exps, seg_begin):
    """Homomorphic sums of consecutive segments: segment s covers
    [seg_begin[s], seg_begin[s+1]); result exponent = min exponent of the
    segment (paillier.py:106-123 folded; order-free)."""
    dk = ctx.device_key()
    seg = np.ascontiguousarray(seg_begin, dtype=np.int64)
    nseg = seg.shape[0] - 1
    n = len(raws)
    e = np.asarray(exps, dtype=np.int64)
    emin = np.zeros(nseg, dtype=np.int64)
    d = np.zeros(n, dtype=np.int32)
    for s in range(nseg):
        lo, hi = int(seg[s]), int(seg[s + 1])
        if hi > lo:
            emin[s] = e[lo:hi].min()
            d[lo:hi] = (e[lo:hi] - emin[s]).astype(np.int32)
    dmax = int(d.max()) if n else 0
    cw = nat.ints_to_words(raws, dk.n2w) if n else np.zeros((1, dk.n2w), dtype=np.uint32)
    out = np.empty((nseg, dk.n2w), dtype=np.uint32)
    nat.check(nat.lib().xhe_segprod_host(dk.handle, _vp(cw), _vp(d), dmax, n, _vp(seg), nseg, _vp(out)), "segprod")
    return nat.words_to_ints(out), emin
