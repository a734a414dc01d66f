"""Batched device operations behind the drop-in API, on flat word buffers.

Ciphertexts travel as C-contiguous uint32 [count, n2w] little-endian words
plus int32 [count] exponents (the PaillierArray layout, include/xhe.h); the
`*_words` functions take and return those buffers and never build Python
ints. The int-list forms at the bottom serve single-element operations
(PaillierCiphertext) and convert at the edge.

Element-independent operations (encrypt, decrypt, add, scalar mul,
obfuscate) are split over the context's shard devices (PaillierContext.
shard_devices: num_cores / $XHE_DEVICES, the reference's process pool,
paillier.py:321-332,388-394): contiguous element ranges, one host thread and
one key handle per device, each writing its own slice of the output. There is
no CPU arithmetic path: a missing library or GPU raises from xfl_amd._native.
"""
import concurrent.futures
import ctypes
import itertools
import os
import threading

import numpy as np

from .. import _native as nat

_nonce = itertools.count(1)
_nonce_lock = threading.Lock()
_pool = None
MIN_SHARD = 1 << 16  # elements per device below which a call stays on one device


def _seed():
    with _nonce_lock:
        n = next(_nonce)
    return os.urandom(32), n


def _u32(a):
    return np.ascontiguousarray(a, dtype=np.uint32)


def _i32(a):
    return np.ascontiguousarray(a, dtype=np.int32)


def _vp(a, row=0):
    """pointer to row `row` of a C-contiguous array (None for None)"""
    if a is None:
        return None
    return ctypes.c_void_p(a.ctypes.data + row * (a.strides[0] if a.ndim else 0))


def _executor():
    global _pool
    if _pool is None:
        _pool = concurrent.futures.ThreadPoolExecutor(max_workers=16, thread_name_prefix="xhe-shard")
    return _pool


def sharded(ctx, count, body, num_cores=-1):
    """Run body(device_key, lo, hi) over contiguous slices of [0, count), one
    slice per shard device (ctypes releases the GIL, so the devices run
    concurrently). Small batches stay on the first device."""
    devs = ctx.shard_devices(num_cores)
    k = max(1, min(len(devs), count // MIN_SHARD))
    if k == 1:
        body(ctx.device_key(devs[0]), 0, count)
        return
    keys = [ctx.device_key(d) for d in devs[:k]]  # built here, not concurrently
    bounds = [count * i // k for i in range(k + 1)]
    futs = [_executor().submit(body, keys[i], bounds[i], bounds[i + 1]) for i in range(k)]
    for f in futs:
        f.result()


def nw_of(ctx):
    """32-bit words of m (the device key's nw: key size class of n / 32)"""
    from .context import device_key_bits
    return device_key_bits(ctx.n) // 32


def n2w_of(ctx):
    """32-bit words of a ciphertext (the device key's n2w)"""
    return 2 * nw_of(ctx)


# ------------------------------------------------------------ encryption
def encrypt_floats_words(ctx, xs, precision, max_exponent, obfuscation, num_cores=-1):
    """Paillier.encrypt over float64 values (paillier.py:273-339): device
    encode + ChaCha20 draws + encrypt -> (ct words, exponents, status)."""
    x = np.ascontiguousarray(xs, dtype=np.float64).reshape(-1)
    n = x.shape[0]
    n2w = n2w_of(ctx)
    ct = nat.empty((n, n2w), np.uint32)
    ex = np.empty(n, dtype=np.int32)
    st = np.empty(n, dtype=np.int32)
    if n == 0:
        return ct, ex, st
    prec = -1 if precision is None else int(precision)
    has_max = max_exponent is not None
    if obfuscation:
        ctx.note_encrypt_volume(n)

    def body(dk, lo, hi):
        seed, nonce = _seed()  # fresh draws per shard
        nat.check(nat.lib().xhe_encrypt_f64_host(dk.handle, _vp(x, lo), hi - lo, prec, int(has_max),
                                                 int(max_exponent) if has_max else 0, int(bool(obfuscation)),
                                                 seed, nonce, _vp(ct, lo), _vp(ex, lo), _vp(st, lo)), "encrypt")
    sharded(ctx, n, body, num_cores)
    return ct, ex, st


def encrypt_encoded_words(ctx, mw, obfuscation, num_cores=-1):
    """encrypt already-encoded integers m (0 <= m < n, nw words each)."""
    mw = _u32(mw)
    n = mw.shape[0]
    ct = nat.empty((n, n2w_of(ctx)), np.uint32)
    if n == 0:
        return ct
    if obfuscation:
        ctx.note_encrypt_volume(n)

    def body(dk, lo, hi):
        seed, nonce = _seed()
        nat.check(nat.lib().xhe_encrypt_words_host(dk.handle, _vp(mw, lo), hi - lo, int(bool(obfuscation)), seed,
                                                   nonce, _vp(ct, lo)), "encrypt")
    sharded(ctx, n, body, num_cores)
    return ct


def obfuscate_words(ctx, cw, num_cores=-1):
    """PaillierCiphertext.obfuscate for a batch: c * X, X a fresh obfuscator
    (an encryption of 0), paillier.py:189-232."""
    cw = _u32(cw)
    n = cw.shape[0]
    if n == 0:
        return cw.copy()
    xs = encrypt_encoded_words(ctx, np.zeros((n, nw_of(ctx)), dtype=np.uint32), True, num_cores)
    z = np.zeros(n, dtype=np.int32)
    return add_words(ctx, cw, z, xs, z, num_cores)[0]


# ------------------------------------------------------------ decryption
def decrypt_words(ctx, cw, num_cores=-1):
    """decrypt -> encoded m words (paillier.py:347-365)."""
    cw = _u32(cw)
    n = cw.shape[0]
    out = np.empty((n, nw_of(ctx)), dtype=np.uint32)
    if n == 0:
        return out

    def body(dk, lo, hi):
        nat.check(nat.lib().xhe_decrypt_host(dk.handle, _vp(cw, lo), hi - lo, _vp(out, lo)), "decrypt")
    sharded(ctx, n, body, num_cores)
    return out


def decrypt_decode_words(ctx, cw, exps, num_cores=-1, want_m=False):
    """decrypt + decode + float32 on the device -> (f64, f32, status[, m])
    (paillier.py:370-398, encoder.py:56-64)."""
    cw = _u32(cw)
    e = _i32(exps)
    n = cw.shape[0]
    f64 = np.empty(n, dtype=np.float64)
    f32 = np.empty(n, dtype=np.float32)
    st = np.empty(n, dtype=np.int32)
    m = np.empty((n, nw_of(ctx)), dtype=np.uint32) if want_m else None
    if n:
        def body(dk, lo, hi):
            nat.check(nat.lib().xhe_decrypt_decode_host(dk.handle, _vp(cw, lo), _vp(e, lo), hi - lo, _vp(f64, lo),
                                                        _vp(f32, lo), _vp(st, lo), _vp(m, lo)), "decrypt")
        sharded(ctx, n, body, num_cores)
    return (f64, f32, st, m) if want_m else (f64, f32, st)


# ------------------------------------------------------------ homomorphic ops
def add_words(ctx, aw, ea, bw, eb, num_cores=-1):
    """ciphertext + ciphertext with exponent alignment (paillier.py:79-123)
    -> (words, exponents)."""
    aw, bw = _u32(aw), _u32(bw)
    ea, eb = _i32(ea), _i32(eb)
    n = aw.shape[0]
    out = nat.empty(aw.shape, np.uint32)
    eo = np.empty(n, dtype=np.int32)
    if n == 0:
        return out, eo
    dmax = int(np.max(np.abs(ea.astype(np.int64) - eb.astype(np.int64))))

    def body(dk, lo, hi):
        nat.check(nat.lib().xhe_mulmod_host(dk.handle, _vp(aw, lo), _vp(ea, lo), _vp(bw, lo), _vp(eb, lo), hi - lo,
                                            dmax, _vp(out, lo), _vp(eo, lo)), "add")
    sharded(ctx, n, body, num_cores)
    return out, eo


def powmod_words(ctx, cw, kw_, kbits, invert_first=False, num_cores=-1):
    """c^k (or (c^-1)^k) mod n^2 per element; k as [count, kw] words."""
    cw = _u32(cw)
    kw_ = _u32(kw_)
    n = cw.shape[0]
    out = nat.empty(cw.shape, np.uint32)
    if n == 0:
        return out
    kwords = kw_.shape[1]

    def body(dk, lo, hi):
        nat.check(nat.lib().xhe_powmod_host(dk.handle, _vp(cw, lo), _vp(kw_, lo), kwords, int(kbits), hi - lo,
                                            int(bool(invert_first)), _vp(out, lo)), "powmod")
    sharded(ctx, n, body, num_cores)
    return out


def raw_mul_words(ctx, cw, kabs, neg, num_cores=-1):
    """PaillierCiphertext._raw_mul (paillier.py:156-187) for encoded scalars
    given as |k| with a sign: a positive k gives c^k; a negative scalar
    (encoded n - |k|, >= min_value_for_negative) gives inv(c)^|k|.
    kabs: int64 array (|k| < 2^63) or [count, kw] uint32 words."""
    cw = _u32(cw)
    n = cw.shape[0]
    out = np.empty_like(cw)
    if n == 0:
        return out
    kw_, kbits = _scalar_words(kabs, n)
    neg = np.asarray(neg, dtype=bool).reshape(-1)
    for flag in (False, True):
        idx = np.nonzero(neg == flag)[0]
        if idx.size == 0:
            continue
        if idx.size == n:
            out[:] = powmod_words(ctx, cw, kw_, kbits, flag, num_cores)
        else:
            out[idx] = powmod_words(ctx, cw[idx], kw_[idx], kbits, flag, num_cores)
    return out


def _scalar_words(kabs, n):
    """|k| (int64 array or [n, kw] uint32 words) -> (words, bit length)"""
    if isinstance(kabs, np.ndarray) and kabs.ndim == 1:
        kabs = np.ascontiguousarray(kabs, dtype=np.uint64)
        return kabs.view(np.uint32).reshape(n, 2), max(1, int(kabs.max()).bit_length())
    kw_ = _u32(kabs)
    return kw_, (max(1, max(nat.words_to_ints(kw_)).bit_length()) if n else 1)


def raw_mul_dev(dk, d, kabs, neg):
    """raw_mul_words on device words (resident.py): c^|k|, or inv(c)^|k| for
    the negative branch, per element -> device words"""
    from . import resident
    n = d.shape[0]
    kw_, kbits = _scalar_words(kabs, n)
    neg = np.asarray(neg, dtype=bool).reshape(-1)
    if not neg.any() or neg.all():
        return resident.powmod(dk, d, kw_, kbits, bool(neg[0]))
    out = resident.empty(dk.device, tuple(d.shape))
    for flag in (False, True):
        idx = np.nonzero(neg == flag)[0]
        resident.put_rows(out, idx, resident.powmod(dk, resident.take(d, idx), kw_[idx], kbits, flag))
    return out


def gap_threshold(ctx):
    """Smallest alignment gap d with 1 << d >= min_value_for_negative: from
    there on _decrease_exponent_to's scalar takes _raw_mul's negative branch,
    c^(2^d - n) instead of c^(2^d) (paillier.py:79-86, 173-187)."""
    return (int(ctx.min_value_for_negative) - 1).bit_length()


def gap_power(ctx, D, bigs):
    """The power a leaf of an addition tree ends up raised to when the
    alignment shifts along its path sum to D and the ones in `bigs` took the
    negative branch: exponents multiply along the path, each shift s
    contributing 2^s, or 2^s - n when s >= gap_threshold."""
    n = int(ctx.n)
    E = 1 << (D - sum(bigs))
    for s in bigs:
        E *= (1 << s) - n
    return E


def fold_gap_powers(ctx, exps, seg_begin):
    """Leaves of LEFT FOLDS (((x0 + x1) + x2) + ..., numpy's object-array
    add.reduce and Python's sum) whose path crosses a negative-branch gap:
    {leaf index: power} (gap_power). At step k the accumulator (exponent m =
    min so far) meets x_k: x_k is aligned by e_k - m if larger, else every
    leaf so far by m - e_k. Only segments whose exponent range reaches the
    threshold are walked."""
    dneg = gap_threshold(ctx)
    seg = np.asarray(seg_begin, dtype=np.int64)
    e = np.asarray(exps, dtype=np.int64).reshape(-1)
    out = {}
    if e.size == 0:
        return out
    lens = np.diff(seg)
    nz = np.nonzero(lens > 0)[0]
    rng = np.maximum.reduceat(e, seg[:-1][nz]) - np.minimum.reduceat(e, seg[:-1][nz])
    for s in nz[rng >= dneg]:
        lo, hi = int(seg[s]), int(seg[s + 1])
        ev = [int(v) for v in e[lo:hi]]
        m = ev[0]
        own, drops = {}, []   # own[k]: x_k's own big shift; drops: (k, acc's big shift at step k)
        for k in range(1, len(ev)):
            if ev[k] - m >= dneg:
                own[k] = ev[k] - m
            elif m - ev[k] >= dneg:
                drops.append((k, m - ev[k]))
            m = min(m, ev[k])
        # one reverse pass: the drops at steps k > i as a running (count, shift
        # sum, product of (2^s - n)), i.e. gap_power's factors without
        # rebuilding the list per leaf
        n = int(ctx.n)
        dk = {k: d for k, d in drops}
        cnt, ssum, prod = 0, 0, 1
        for i in range(len(ev) - 1, -1, -1):
            if i + 1 in dk:
                d = dk[i + 1]
                cnt, ssum, prod = cnt + 1, ssum + d, prod * ((1 << d) - n)
            if i in own or cnt:
                o = own.get(i)
                ps, pp = (ssum + o, prod * ((1 << o) - n)) if o is not None else (ssum, prod)
                out[lo + i] = (1 << (ev[i] - m - ps)) * pp
    return out


def pow_signed_words(ctx, cw, powers):
    """c_i^E_i mod n^2 for Python-int powers of either sign (a negative power
    inverts first): the device's _raw_mul branches (paillier.py:173-187)."""
    kabs = [abs(int(E)) for E in powers]
    kw = max(1, (max(k.bit_length() for k in kabs) + 31) // 32)
    return raw_mul_words(ctx, cw, nat.ints_to_words(kabs, kw), np.array([E < 0 for E in powers], dtype=bool))


def segment_sums_words(ctx, cw, exps, seg_begin, gap_powers=None, fold=False):
    """Homomorphic sums of consecutive segments: segment s covers
    [seg_begin[s], seg_begin[s+1]); result exponent = min exponent of the
    segment (paillier.py:106-123 folded; order-free). An empty
    segment gives 1 with exponent 0.

    Past the negative-branch gap (gap_threshold) the reference's bits depend on
    the addition tree: gap_powers {leaf: power} (gap_power) gives those
    leaves' final powers, or fold=True derives them for left folds of each
    segment in input order (fold_gap_powers); such leaves are raised to their
    power first and enter the product unaligned."""
    cw = _u32(cw)
    seg, emin, d, gap_powers = _segment_plan(ctx, cw.shape[0], exps, seg_begin, gap_powers, fold)
    if gap_powers:
        idx = np.fromiter(gap_powers.keys(), dtype=np.int64, count=len(gap_powers))
        cw = cw.copy()
        cw[idx] = pow_signed_words(ctx, cw[idx], [gap_powers[int(i)] for i in idx])
        d[idx] = 0
    return segprod_words(ctx, cw, d, seg), emin.astype(np.int32)


def _segment_plan(ctx, n, exps, seg_begin, gap_powers, fold):
    """(offsets, per-segment min exponent, per-element shift d, gap powers)"""
    seg = np.ascontiguousarray(seg_begin, dtype=np.int64)
    nseg = seg.shape[0] - 1
    e = np.asarray(exps, dtype=np.int64).reshape(-1)
    lens = np.diff(seg)
    emin = np.zeros(nseg, dtype=np.int64)
    nz = lens > 0
    if n:
        emin[nz] = np.minimum.reduceat(e, seg[:-1][nz])
    d = (e - np.repeat(emin, lens)).astype(np.int32)
    if fold and n and gap_powers is None:
        gap_powers = fold_gap_powers(ctx, e, seg)
    return seg, emin, d, gap_powers


def segment_sums_dev(ctx, dk, cd, exps, seg_begin, gap_powers=None, fold=False):
    """segment_sums_words on device words -> (device [nseg, n2w], emin)"""
    from . import resident
    seg, emin, d, gap_powers = _segment_plan(ctx, cd.shape[0], exps, seg_begin, gap_powers, fold)
    if gap_powers:
        idx = np.fromiter(gap_powers.keys(), dtype=np.int64, count=len(gap_powers))
        powers = [gap_powers[int(i)] for i in idx]
        kabs = [abs(int(E)) for E in powers]
        kw = max(1, (max(k.bit_length() for k in kabs) + 31) // 32)
        cd = resident.clone(cd)
        resident.put_rows(cd, idx, raw_mul_dev(dk, resident.take(cd, idx), nat.ints_to_words(kabs, kw),
                                               np.array([E < 0 for E in powers], dtype=bool)))
        d[idx] = 0
    return resident.segprod(dk, cd, d, seg), emin.astype(np.int32)


def segprod_words(ctx, cw, d, seg):
    """out[s] = prod_{i in segment s} c_i^(2^d_i) mod n^2: one xhe_segprod
    call (int32 d >= 0, int64 seg offsets)."""
    n = cw.shape[0]
    nseg = seg.shape[0] - 1
    dmax = int(d.max()) if n else 0
    n2w = n2w_of(ctx)
    src = cw if n else np.zeros((1, n2w), dtype=np.uint32)
    d = _i32(d)
    out = np.empty((nseg, n2w), dtype=np.uint32)
    dk = ctx.device_key(ctx.own_device())  # the process's GPU, as _run and the resident path use
    nat.check(nat.lib().xhe_segprod_host(dk.handle, _vp(src), _vp(d) if dmax else None, dmax, n, _vp(seg), nseg,
                                         _vp(out)), "segprod")
    return out


def multiexp_words(ctx, bw, idx, kw_, kbits, win_bits=0):
    """out[j] = prod_t bases[idx[j][t]]^k[j][t] mod n^2 (k >= 0, [ncols,
    nterms, kw] words): one xhe_multiexp call (Straus windows, per-base tables
    shared by all j)."""
    bw = _u32(bw)
    iw = np.ascontiguousarray(idx, dtype=np.int32)
    ncols, nterms = iw.shape
    kw_ = _u32(kw_).reshape(ncols * nterms, -1)
    if ncols == 0 or nterms == 0 or bw.shape[0] == 0:
        raise ValueError("multiexp: empty problem")
    out = np.empty((ncols, n2w_of(ctx)), dtype=np.uint32)
    dk = ctx.device_key(ctx.own_device())
    nat.check(nat.lib().xhe_multiexp_host(dk.handle, _vp(bw), bw.shape[0], _vp(iw), _vp(kw_), kw_.shape[1],
                                          int(kbits), ncols, nterms, int(win_bits), _vp(out)), "multiexp")
    return out


# ------------------------------------------------------------ int forms
def encrypt_floats(ctx, xs, precision, max_exponent, obfuscation):
    """-> (raw ints, exponents, status)"""
    ct, ex, st = encrypt_floats_words(ctx, xs, precision, max_exponent, obfuscation)
    return (nat.words_to_ints(ct) if ct.shape[0] else []), ex, st


def encrypt_encoded(ctx, ms, obfuscation):
    if len(ms) == 0:
        return []
    return nat.words_to_ints(encrypt_encoded_words(ctx, nat.ints_to_words(ms, nw_of(ctx)), obfuscation))


def decrypt_ints(ctx, raws):
    if len(raws) == 0:
        return []
    return nat.words_to_ints(decrypt_words(ctx, nat.ints_to_words(raws, n2w_of(ctx))))


def decrypt_float32(ctx, raws, exps):
    """-> (f64, f32, status)"""
    n2w = n2w_of(ctx)
    cw = nat.ints_to_words(raws, n2w) if len(raws) else np.zeros((0, n2w), dtype=np.uint32)
    return decrypt_decode_words(ctx, cw, exps)


def add(ctx, ra, ea, rb, eb):
    if len(ra) == 0:
        return [], np.empty(0, dtype=np.int32)
    n2w = n2w_of(ctx)
    out, eo = add_words(ctx, nat.ints_to_words(ra, n2w), ea, nat.ints_to_words(rb, n2w), eb)
    return nat.words_to_ints(out), eo


def powmod(ctx, raws, ks, invert_first=False):
    if len(raws) == 0:
        return []
    kbits = max(int(k).bit_length() for k in ks)
    kw = max(1, (kbits + 31) // 32)
    out = powmod_words(ctx, nat.ints_to_words(raws, n2w_of(ctx)), nat.ints_to_words(ks, kw), kbits, invert_first)
    return nat.words_to_ints(out)


def raw_mul(ctx, raws, ks):
    """_raw_mul (paillier.py:156-187) for k >= 0: c^(k - n) when k >=
    min_value_for_negative (inv(c)^(n - k) for k < n; _decrease_exponent_to's
    1 << d may exceed n, and then the power k - n is positive), else c^k."""
    n = len(raws)
    if n == 0:
        return []
    thr = ctx.min_value_for_negative
    return nat.words_to_ints(pow_signed_words(ctx, nat.ints_to_words(raws, n2w_of(ctx)),
                                              [int(k) - ctx.n if k >= thr else int(k) for k in ks]))


def obfuscate(ctx, raws):
    if len(raws) == 0:
        return []
    return nat.words_to_ints(obfuscate_words(ctx, nat.ints_to_words(raws, n2w_of(ctx))))


def segment_sums(ctx, raws, exps, seg_begin, gap_powers=None):
    n2w = n2w_of(ctx)
    cw = nat.ints_to_words(raws, n2w) if len(raws) else np.zeros((0, n2w), dtype=np.uint32)
    out, emin = segment_sums_words(ctx, cw, exps, seg_begin, gap_powers=gap_powers)
    return nat.words_to_ints(out), emin


def multiexp(ctx, bases, idx, ks, win_bits=0):
    flat_k = [int(k) for row in ks for k in row]
    kbits = max(1, max(k.bit_length() for k in flat_k))
    kw = (kbits + 31) // 32
    ncols = len(idx)
    out = multiexp_words(ctx, nat.ints_to_words(bases, n2w_of(ctx)), np.asarray(idx, dtype=np.int32).reshape(ncols, -1),
                         nat.ints_to_words(flat_k, kw), kbits, win_bits)
    return nat.words_to_ints(out)
