"""Throughput benchmark: 2048-bit Paillier encryptions/s, device-resident.

One step = the label-trainer encryption of one synthetic batch
(logistic_regression/label_trainer.py:193-197 at BASELINE config 2 size):
    encode float64 -> m (precision 7)   (encoder.py:29-54)
    draw DJN obfuscation exponents a   (paillier.py:195, device ChaCha20)
    c = (1 + n m) h^a mod n^2 via CRT  (paillier.py:189-209, 283)
for N elements per GPU that are already resident in HBM. With --gpus > 1 each
rank encrypts its own shard (weak scaling) and the step ends with an RCCL
all-gather of the ciphertext shards over xGMI, so every rank holds the whole
vector (the reassembly step of SURVEY.md 8(e)).

    python bench.py [--gpus N --steps K --warmup W --n ELEMENTS]
"""
import argparse
import json
import math
import os
import random
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

PEAK_MAC_PER_S = 1024 * 16 * 2.4e9  # v_mad_u64_u32: 4 cycles/wave64 on 1024 SIMDs at 2.4 GHz (tools/microbench)


def make_key(bits, seed):
    """Deterministic DJN key (context.py:73-84 / :123-150 with a seeded RNG)."""
    from xfl_amd.paillier.utils import getprimeover
    rng = random.Random(seed)
    while True:
        p = getprimeover(bits // 2, rng=rng)
        q = getprimeover(bits // 2, rng=rng)
        if p != q and math.gcd(p - 1, q - 1) == 2:
            break
    n = p * q
    x = rng.getrandbits(n.bit_length()) | (1 << (n.bit_length() - 1))
    h_pow_n = pow(-(x * x), n, n * n)
    return p, q, n, h_pow_n


def algorithmic_macs_per_element(bits, win_bits, rand_bits):
    """32-bit-limb MACs of the fixed-base DJN-CRT encryption (SURVEY 8(d) model):
    per prime 1 (n m R) + nwin table products + 1 (from Montgomery) CIOS
    products of s = bits/32 limbs at 2s^2+s MACs each; plus the CRT product and
    the q^2 * h wide multiply (s^2). Second value: the table products alone
    (the dominant kernel's model work)."""
    from xfl_amd._native import win_layout
    s = bits // 32
    nwin, _ = win_layout(rand_bits, win_bits)
    prod = 2 * s * s + s
    return 2 * (nwin + 2) * prod + prod + s * s, 2 * nwin * prod


def cpu_baseline(bits, seconds, cores):
    """The reference algorithm timed on this host for a bounded sample:
    preferably the C port on GMP's mpz_powm (what gmpy2 calls; oracle/
    gmp_baseline.c, dlopen libgmp.so.10) over `cores` threads, else the
    pure-Python restatement (oracle/paillier_oracle.py) over `cores` processes."""
    import multiprocessing as mp
    from oracle import bench_cpu
    try:
        r = bench_cpu.gmp_rate(bits, seconds, cores)
    except Exception:
        r = None
    if r is not None:
        total, wall = r
        return {"value": total / wall, "unit": "encrypts/s", "cores": cores, "kind": "port",
                "sample": f"{total} DJN-CRT private-key encryptions (2 mpz_powm mod p^2/q^2 + CRT + mulmod, "
                          f"precision-7 encode), {cores} threads x ~{seconds:.0f}s, C port on system GMP "
                          "(oracle/gmp_baseline.c) - same GMP routines as the reference's gmpy2"}
    with mp.get_context("fork").Pool(cores) as pool:
        t0 = time.time()
        counts = pool.map(bench_cpu.encrypt_for, [(bits, seconds, i) for i in range(cores)])
        wall = time.time() - t0
    total = sum(counts)
    return {"value": total / wall, "unit": "encrypts/s", "cores": cores, "kind": "port",
            "sample": f"{total} DJN-CRT private-key encryptions of float64 plaintexts (precision 7), "
                      f"{cores} worker processes x ~{seconds:.0f}s, pure-Python pow (oracle/bench_cpu.py)"}


TABLE_ROW_BYTES = {2048: 256, 3072: 384, 4096: 512, 8192: 1024}  # packed rows: K/32 words x 4 (xhe.hip Shape<K>::RW)


def table_bytes(bits, win_bits):
    """Device bytes of the two fixed-base tables (xhe_key_create, include/xhe.h)."""
    from xfl_amd._native import table_bytes as tb
    return tb(bits, win_bits)


def pick_window(bits, free_bytes, margin=16 << 30, split=False):
    """The window layout with the fewest table products per element whose
    tables leave `margin` of HBM free (ties: fewer bytes): uniform w <= 24,
    and with split=True also split w <= 23 (include/xhe.h XHE_WIN_SPLIT).
    Split layouts are not the default: at 2048 bits 23s (44 products, 240 GB)
    measured only 1.0 % faster than 23 (45, 193 GB) - its 2^24-row windows
    cost more per random row - for 25 % more table memory and build time."""
    from xfl_amd._native import XHE_WIN_SPLIT, win_layout
    best = None
    for w in range(12, 25):
        for wb in (w, w | XHE_WIN_SPLIT) if split and w <= 23 else (w,):
            nb = table_bytes(bits, wb)
            if nb + margin > free_bytes:
                continue
            key = (win_layout(bits // 2, wb)[0], nb)
            if best is None or key < best[0]:
                best = (key, wb)
    return best[1] if best else 12


def pmc_traffic(win_bits, n, kernel="k_djn_pmd"):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC passes
    (tools/profile_box.sh -> tools/pmc_traffic.py), when they were taken on
    this configuration; else None. Counters cannot be read inside this run
    (rocprofv3 --pmc is its own pass). The newest round's file wins (the
    kernel changed between rounds; before round 4 the files were named after
    the k_djn_pow label)."""
    from xfl_amd._native import win_spec
    for rnd, name in (("r6", kernel), ("r5", kernel), ("r4", kernel), ("r3", "k_djn_pow"), ("r2", "k_djn_pow")):
        if name != kernel:  # an older round's pass measured another kernel: not this one's traffic
            continue
        path = os.path.join(ROOT, "profiles", rnd, f"{name}_pmc.json")
        try:
            with open(path) as f:
                rec = json.load(f)
        except (OSError, ValueError):
            continue
        if rec.get("kernel", kernel) != kernel:
            continue
        if str(rec.get("win")) != win_spec(win_bits) or rec.get("n") != n or "traffic_bytes" not in rec:
            return None, None, None
        return rec["traffic_bytes"], os.path.relpath(path, ROOT), rec
    return None, None, None


def sliding_window_ops(e, w=5):
    """(squarings, products) of the kernels' wave-uniform sliding-window
    schedule for the exponent e (pow_uniform_exp / pmd_pow_uniform): the
    table x, x^3 .. x^31 (one squaring, 15 products), the first window's odd
    power as the start value, then per zero bit a squaring and per window
    [i..j] its i - j + 1 squarings and one product"""
    bits = bin(e)[2:]
    sq, mul = 1, 2 ** (w - 1) - 1
    i = 0
    i += min(w, len(bits))
    while i and bits[i - 1] == "0":  # the window ends in a set bit
        i -= 1
    while i < len(bits):
        if bits[i] == "0":
            sq += 1
            i += 1
            continue
        j = min(len(bits), i + w)
        while bits[j - 1] == "0":
            j -= 1
        sq += j - i
        mul += 1
        i = j
    return sq, mul


def barrett_add_mads():
    """v_mad_u64_u32 lane-instructions per element of k_add_barrett
    (barrett_dev.hpp): every round walks the union of its 32 columns' terms
    in pairs of 4-term blocks, 8 lanes x 4 columns"""
    S, RC = 152, 32

    def cols(C0, LX, LY):
        ilo = max(0, C0 - (LY - 1))
        ihi = min(LX - 1, C0 + RC - 1)
        ib0 = ilo & ~3
        return ((ihi + 1 - ib0 + 7) >> 3) * 8 * 4 * 8  # npair pairs x 8 terms x 4 columns x 8 lanes
    a = sum(cols(RC * r, S, S) for r in range((2 * S + RC - 1) // RC))
    b0 = S - 4
    b = sum(cols(b0 + RC * r, S + 1, S + 1) for r in range((2 * S + 2 - b0 + RC - 1) // RC))
    c = sum(cols(RC * r, S + 1, S) for r in range((S + 1 + RC - 1) // RC))
    return a + b + c


def issued_mads(bits, key_material, win_bits):
    """v_mad_u64_u32 lane-instructions per operation from each kernel's
    schedule (digit product 5 K^2, digit squaring 4 K^2 at K = 37
    mod P^2 (28-bit limbs) and K = 80 mod n^2 (27-bit); Montgomery product
    2 S^2 at S = 74 mod P^2 and S = 152 mod n^2), for the 2048-bit kernels
    the ops figures time; the dominant kernel of each operation, conversions
    and CRT left out (a lower bound on what was issued)"""
    if bits != 2048:
        return {}
    p, q, n, _ = key_material
    from xfl_amd import _native as nat
    dsq, dmul, nsq, nmul, mp2, mn2 = 4 * 37 ** 2, 5 * 37 ** 2, 4 * 80 ** 2, 5 * 80 ** 2, 2 * 74 ** 2, 2 * 152 ** 2
    rand_bits = n.bit_length() // 2
    out = {}
    nwin = nat.win_layout(rand_bits, win_bits)[0]
    out["headline"] = 2 * ((nwin - 1) * dmul + 37 ** 2 + 2 * mp2)  # k_djn_pmd: table products, to_mont2, (1 + n m)
    sp, mp = sliding_window_ops(p - 1)
    sq_, mq = sliding_window_ops(q - 1)
    out["decrypt_per_s"] = (sp + sq_) * dsq + (mp + mq) * dmul  # k_dec_pmd_pow, x^(P-1) per prime
    out["add_per_s"] = barrett_add_mads()
    out["sum_per_s"] = int(1.035 * mn2)  # k_chunk_prod_words: ~1 product per element (+1 per chunk, upper levels)
    out["encrypt_public_djn_per_s"] = (nat.win_layout(rand_bits, 16)[0] - 1) * nmul  # k_djn_pub_nd at window 16
    s, m = sliding_window_ops(n)
    out["encrypt_public_nodjn_per_s"] = s * nsq + m * nmul  # k_ndig_pow_n: r^n
    ep, eq = n % (p * (p - 1)), n % (q * (q - 1))
    sp, mp = sliding_window_ops(ep)
    sq_, mq = sliding_window_ops(eq)
    out["encrypt_private_nodjn_per_s"] = (sp + sq_) * dsq + (mp + mq) * dmul  # k_dec_pmd_pow with e_P
    out["scalar_mul_53bit_per_s"] = 53 * nsq + 26 * nmul  # k_ndig_pow_k: 4-bit windows, table x^2..x^15
    return out


def model_macs(bits, key_material, win_bits):
    """SURVEY 8(d)'s 32-bit CIOS model per operation (2 s^2 + s MACs per
    product, s = K/32 words per prime, 2 s per n^2): what roofline.achieved
    uses for the headline"""
    if bits != 2048:
        return {}
    p, q, n, _ = key_material
    from xfl_amd import _native as nat
    s1, s2 = 64, 128
    prod1, prod2 = 2 * s1 * s1 + s1, 2 * s2 * s2 + s2
    nwin = nat.win_layout(n.bit_length() // 2, win_bits)[0]
    vb = lambda e: e.bit_length() + -(-e.bit_length() // 5) + 16  # noqa: E731  variable-base window-5 products
    ep, eq = n % (p * (p - 1)), n % (q * (q - 1))
    return {"headline": 2 * nwin * prod1, "decrypt_per_s": (vb(p - 1) + vb(q - 1)) * prod1, "add_per_s": prod2,
            "sum_per_s": prod2, "encrypt_public_djn_per_s": nat.win_layout(n.bit_length() // 2, 16)[0] * prod2,
            "encrypt_public_nodjn_per_s": vb(n) * prod2, "encrypt_private_nodjn_per_s": (vb(ep) + vb(eq)) * prod1,
            "scalar_mul_53bit_per_s": (53 + 11 + 16) * prod2}


def issued_fractions(ops, bits, key_material, win_bits, headline_rate, clock_ghz):
    """ops["issued"]: per operation the schedule's mads x the measured rate
    over the v_mad_u64_u32 issue peak (16,384 lanes x clock: 2.4 GHz, and
    the clock the counter passes measured under this load), next to the
    8(d) model fraction"""
    mads, model = issued_mads(bits, key_material, win_bits), model_macs(bits, key_material, win_bits)
    rates = dict(ops)
    rates["headline"] = headline_rate
    out = {}
    for k, v in mads.items():
        r = rates.get(k)
        if not r:
            continue
        rec = {"mads_per_op": v, "model_macs_per_op": model.get(k), "rate_per_s": r,
               "issued_mad_frac": v * r / PEAK_MAC_PER_S, "model_frac": model.get(k, 0) * r / PEAK_MAC_PER_S}
        if clock_ghz:
            rec["issued_mad_frac_at_clock"] = v * r / (16384 * clock_ghz * 1e9)
        out[k] = rec
    return out


def _timed(fn, reps=3):
    """Average seconds per call of fn() on the current stream (1 untimed warm call)."""
    import torch
    fn()
    torch.cuda.synchronize()
    t0 = time.time()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.time() - t0) / reps


def measure_ops(nat, L, dk, x, m, ex, ct, rnd, N, stream, key_material):
    """Rates of the other operations on the path (BASELINE configs 2, 3, 5),
    device-resident except where named; plus the host-buffer (PCIe-inclusive)
    encrypt/decrypt rates. Each is checked where a cheap property exists."""
    import ctypes
    import torch
    out = {}
    # config 2: decrypt the step's ciphertexts; round trip must give back m exactly
    m2 = torch.empty_like(m)
    t = _timed(lambda: nat.check(L.xhe_decrypt(dk.handle, ct.data_ptr(), N, m2.data_ptr(), stream), "decrypt"))
    out["decrypt_per_s"] = N / t
    out["roundtrip_bit_exact"] = bool(torch.equal(m, m2))
    # ciphertext add (paillier.py:153-154), equal exponents
    ct2 = torch.empty_like(ct)
    t = _timed(lambda: nat.check(L.xhe_mulmod(dk.handle, ct.data_ptr(), None, ct.data_ptr(), None, N, 0,
                                              ct2.data_ptr(), None, stream), "add"))
    out["add_per_s"] = N / t
    # add with exponent alignment: operands one exponent apart (x * 2^-1 precision shift)
    e1 = torch.zeros(N, dtype=torch.int32, device="cuda")
    e2 = torch.full((N,), -4, dtype=torch.int32, device="cuda")
    t = _timed(lambda: nat.check(L.xhe_mulmod(dk.handle, ct.data_ptr(), e1.data_ptr(), ct.data_ptr(), e2.data_ptr(),
                                              N, 4, ct2.data_ptr(), None, stream), "add_align"))
    out["add_aligned_d4_per_s"] = N / t
    # scalar mul by an encoded float64 (53-bit mantissa, positive branch, paillier.py:156-187)
    nk = min(N, 1 << 18)
    k = torch.randint(0, 1 << 31, (nk, 2), dtype=torch.int64, device="cuda").to(torch.int32)
    k[:, 1] &= (1 << 21) - 1
    k[:, 1] |= 1 << 20
    t = _timed(lambda: nat.check(L.xhe_powmod(dk.handle, ct.data_ptr(), k.data_ptr(), 2, 53, nk, ct2.data_ptr(),
                                              stream), "scalar_mul"))
    out["scalar_mul_53bit_per_s"] = nk / t
    # encrypted mat-vec enc[B] @ X[B, D] at the LR operator's default shape
    # (logistic_regression/trainer.py:166, B = 2048, D = 15): one
    # multi-exponentiation with 60-bit exponents (53-bit mantissas + alignment)
    Bm, Dm = min(N, 2048), 15
    idx = torch.arange(Bm, dtype=torch.int32, device="cuda").repeat(Dm, 1).contiguous()
    kx = torch.randint(0, 1 << 30, (Dm, Bm, 2), dtype=torch.int32, device="cuda")
    kx[..., 1] &= (1 << 28) - 1
    mv = torch.empty((Dm, dk.n2w), dtype=torch.int32, device="cuda")
    t = _timed(lambda: nat.check(L.xhe_multiexp(dk.handle, ct.data_ptr(), Bm, idx.data_ptr(), kx.data_ptr(), 2, 60,
                                                Dm, Bm, 0, mv.data_ptr(), stream), "matvec"))
    out["matvec_2048x15_s"] = t
    out["matvec_terms_per_s"] = Bm * Dm / t
    # config 5: 256-bin histogram of 100k ciphertexts (grad) -> segment products
    ns, nb = min(N, 100_000), 256
    seg = (np.arange(nb + 1, dtype=np.int64) * ns) // nb
    hist = torch.empty((nb, dk.n2w), dtype=torch.int32, device="cuda")
    segp = seg.ctypes.data_as(ctypes.c_void_p)
    t = _timed(lambda: nat.check(L.xhe_segprod(dk.handle, ct.data_ptr(), None, 0, ns, segp, nb, hist.data_ptr(),
                                               stream), "hist"))
    out["hist_256x100k_s"] = t
    # sum of the whole vector (config 3's aggregation)
    one = np.array([0, N], dtype=np.int64)
    t = _timed(lambda: nat.check(L.xhe_segprod(dk.handle, ct.data_ptr(), None, 0, N, one.ctypes.data_as(
        ctypes.c_void_p), 1, hist.data_ptr(), stream), "sum"), reps=2)
    out["sum_per_s"] = N / t
    # the other encryption modes: a remote party holding only
    # the public key (DJN is lost on the wire, context.py:152-168, so it runs
    # r^n mod n^2 with a variable base: paillier.py:228-230), the public DJN
    # form (fixed base mod n^2, paillier.py:210-212) and the private non-DJN
    # CRT form (paillier.py:214-227)
    p_, q_, n_, h_ = key_material
    nm = min(N, 1 << 16)
    rk = torch.empty((nm, dk.nw), dtype=torch.int32, device="cuda")
    ctm = torch.empty((nm, dk.n2w), dtype=torch.int32, device="cuda")
    for tag, args_ in (("encrypt_public_nodjn_per_s", (None, None, None)),
                       ("encrypt_public_djn_per_s", (None, None, h_)),
                       ("encrypt_private_nodjn_per_s", (p_, q_, None))):
        # public DJN at the drop-in's window (a public key's DeviceKey takes the
        # library default, 16: 64 windows of 2^16 rows mod n^2, 2.1 GB)
        k2 = nat.DeviceKey(dk.key_bits, n_, *args_, device=dk.device, win_bits=16 if args_[2] else 0)
        if args_[2]:
            out["encrypt_public_djn_window_bits"] = 16
        nat.check(L.xhe_rand(k2.handle, b"\x01" * 32, 5, nm, rk.data_ptr(), None, stream), "rand")
        t = _timed(lambda: nat.check(L.xhe_encrypt(k2.handle, m.data_ptr(), rk.data_ptr(), nm, ctm.data_ptr(), stream),
                                     tag), reps=2)
        out[tag] = nm / t
        del k2
    # host buffers in and out (PCIe-inclusive), the rate the federated exchange sees
    nh = min(N, 1 << 20)
    xh = x[:nh].cpu().numpy()
    cth = np.empty((nh, dk.n2w), dtype=np.uint32)
    exh = np.empty(nh, dtype=np.int32)
    sth = np.empty(nh, dtype=np.int32)
    vp = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    t = _timed(lambda: nat.check(L.xhe_encrypt_f64_host(dk.handle, vp(xh), nh, 7, 0, 0, 1, os.urandom(32), 7,
                                                        vp(cth), vp(exh), vp(sth)), "encrypt_host"), reps=2)
    out["encrypt_host_buffers_per_s"] = nh / t
    f64 = np.empty(nh, dtype=np.float64)
    f32 = np.empty(nh, dtype=np.float32)
    t = _timed(lambda: nat.check(L.xhe_decrypt_decode_host(dk.handle, vp(cth), vp(exh), nh, vp(f64), vp(f32), vp(sth),
                                                           None), "decrypt_host"), reps=2)
    out["decrypt_decode_host_buffers_per_s"] = nh / t
    out["host_roundtrip_max_abs_err"] = float(np.max(np.abs(f64 - xh)))
    return out


def measure_dropin(nat, device, key_bits, xh, key_material):
    """The same through the drop-in API (what XFL's operators call), with the
    drop-in's own PaillierContext - its window policy (window 16 first, wider
    as the key's encrypted volume grows, context.py WIN_STEPS) and its
    device-resident arrays (xfl_amd/paillier/resident.py): the label trainer's
    Paillier.encrypt(float32[]) -> Paillier.serialize, the receiving side's
    ciphertext_from -> Paillier.decrypt (logistic_regression/label_trainer.py:
    193-199, 258), config 3's pairwise sum, and the LR step's encrypt ->
    np.matmul -> serialize chain (logistic_regression/trainer.py:166). Each
    figure carries the fixed-base window the context's key had after it."""
    import gc
    import torch
    from xfl_amd.paillier import Paillier, PaillierContext
    out = {}
    p_, q_, n_, h_ = key_material
    nh = xh.shape[0]
    # one GPU's rates: pin the drop-in to this rank's GPU
    os.environ["XHE_DEVICES"] = str(device)
    ctx = PaillierContext().init(p_, q_, djn_h_pow_n=h_)
    win = {}

    def note(tag):  # the window of the key the last call used (no rebuild here)
        win[tag] = ctx._dev[device].win_bits
        ctx._volume = 0  # every figure at the fresh context's window (16); the steady state is timed last

    def sync():
        torch.cuda.synchronize()

    x32 = xh.astype(np.float32)
    wire = {}

    def enc_ser(comp):
        wire.pop(comp, None)  # the previous payload is released first, as in a training loop
        wire[comp] = Paillier.serialize(Paillier.encrypt(ctx, x32, precision=7), compression=comp)
    enc = {}

    def enc_only():
        enc.pop(0, None)
        enc[0] = Paillier.encrypt(ctx, x32, precision=7)
        sync()
    out["dropin_encrypt_per_s"] = nh / _timed(enc_only, reps=3)
    note("dropin_encrypt_per_s")
    out["dropin_encrypt_resident"] = bool(enc[0].is_resident)
    ser = {}

    def ser_only():
        ser.pop(0, None)
        enc[0]._st.h = None  # a fresh encryption's words are only in HBM: serialize includes the download
        ser[0] = Paillier.serialize(enc[0], compression=False)
    out["dropin_serialize_per_s"] = nh / _timed(ser_only, reps=3)
    t = _timed(lambda: enc_ser(False), reps=3)
    out["dropin_encrypt_serialize_per_s"] = nh / t
    note("dropin_encrypt_serialize_per_s")
    # config 3's pairwise sum: PaillierArray + PaillierArray on resident operands
    tot = {}

    def add_only():
        tot.pop(0, None)
        tot[0] = enc[0] + enc[0]
        sync()
    out["dropin_add_per_s"] = nh / _timed(add_only, reps=3)
    out["dropin_add_resident"] = bool(tot[0].is_resident and tot[0]._st.h is None)
    # decrypt of a resident array (only the float32 results come back)
    out["dropin_decrypt_resident_per_s"] = nh / _timed(lambda: Paillier.decrypt(ctx, tot[0]), reps=2)
    back2 = Paillier.decrypt(ctx, tot[0])
    out["dropin_add_max_abs_err"] = float(np.max(np.abs(back2 - 2 * x32.astype(np.float64))))
    ser.clear()
    tot.clear()
    gc.collect()
    t = _timed(lambda: Paillier.decrypt(ctx, Paillier.ciphertext_from(None, wire[False], compression=False)), reps=2)
    out["dropin_deserialize_decrypt_per_s"] = nh / t
    t = _timed(lambda: Paillier.ciphertext_from(None, wire[False], compression=False), reps=3)
    out["dropin_deserialize_per_s"] = nh / t
    back = Paillier.decrypt(ctx, Paillier.ciphertext_from(None, wire[False], compression=False))
    out["dropin_roundtrip_max_abs_err"] = float(np.max(np.abs(back - x32)))
    t = _timed(lambda: enc_ser(True), reps=2)
    out["dropin_encrypt_serialize_zstd_per_s"] = nh / t
    note("dropin_encrypt_serialize_zstd_per_s")
    out["wire_bytes_per_ciphertext"] = len(wire[False]) / nh
    # the LR step (B = 2048 residuals, D = 15 features): encrypt -> matmul -> serialize
    rng = np.random.default_rng(11)
    r = rng.standard_normal(2048).astype(np.float32)
    X = rng.standard_normal((2048, 15))
    chain = {}

    def lr_chain():
        chain[0] = Paillier.serialize(Paillier.encrypt(ctx, r, precision=7) @ X)
    out["dropin_chain_encrypt_matmul_serialize_2048x15_s"] = _timed(lr_chain, reps=5)
    got = Paillier.decrypt(ctx, Paillier.ciphertext_from(ctx, chain[0]))
    out["dropin_chain_max_abs_err"] = float(np.max(np.abs(got - r.astype(np.float64) @ X)))
    note("dropin_chain_encrypt_matmul_serialize_2048x15_s")
    out["dropin_table_bytes_w16"] = nat.table_bytes(key_bits, 16)
    out.update(measure_dropin_histogram(ctx))
    # the policy's steady state for a loop of 1 M-element calls: past 64 M
    # encrypted elements the key's tables are rebuilt at window 22 (when they
    # leave 32 GiB free; the rebuild happens in the untimed first call)
    ctx._volume = ctx.WIN_STEPS[-1][0]
    out["dropin_encrypt_steady_per_s"] = nh / _timed(enc_only, reps=3)
    win["dropin_encrypt_steady_per_s"] = ctx._dev[device].win_bits
    # the steady window's ciphertexts decrypt back to the inputs (to the
    # precision-7 encoding and the float32 result)
    back = Paillier.decrypt(ctx, enc[0])
    out["dropin_encrypt_steady_max_abs_err"] = float(np.max(np.abs(back - x32)))
    out["dropin_encrypt_steady_ok"] = bool(np.allclose(back, x32, rtol=1e-6, atol=1e-7))
    # the label trainer's encrypt -> serialize(compression=True) at that window
    out["dropin_encrypt_serialize_zstd_steady_per_s"] = nh / _timed(lambda: enc_ser(True), reps=2)
    win["dropin_encrypt_serialize_zstd_steady_per_s"] = ctx._dev[device].win_bits
    out["dropin_table_bytes_steady"] = nat.table_bytes(key_bits, ctx._dev[device].win_bits)
    out["dropin_window_bits"] = win
    wire.clear()
    enc.clear()
    ctx._dev = {}
    gc.collect()
    torch.cuda.empty_cache()
    return out


def xgb_inputs(n=100_000, nfeat=64, nbins=256):
    """BASELINE config 5's synthetic inputs: g = sigmoid(z) - y,
    h = p (1 - p) (seed 3), bins ~ U{0..255} per feature (seed 4 + f)"""
    import pandas as pd
    rng = np.random.default_rng(3)
    p = 1 / (1 + np.exp(-rng.standard_normal(n)))
    y = rng.integers(0, 2, n)
    g, h = p - y, p * (1 - p)
    values = pd.DataFrame({f"x{f}": np.random.default_rng(4 + f).integers(0, nbins, n).astype(np.uint8)
                           for f in range(nfeat)})
    return g, h, values


def measure_dropin_histogram(ctx, n=100_000, nfeat=64):
    """Config 5 through XFL's own pandas calls: the label side's embed ->
    Paillier.encrypt(precision=0) -> serialize(compression=False), the
    trainer's ciphertext_from -> Feature.create (core/tree/big_feature.py:
    43-46) -> per feature groupby(col)['xfl_grad_hess'].agg({'count', 'sum'})
    (xgboost/decision_tree_trainer.py:151-152) -> res_hist['sum'].to_numpy()
    (:180). Timed: the 64 groupby calls with every bin sum computed (host
    pandas work included), and the same with the operator's to_numpy."""
    import pandas as pd
    import torch
    from xfl_amd.paillier import Paillier
    from xfl_amd.paillier.array import PaillierDtype
    from xfl_amd.paillier_acceleration import embed
    g, h, values = xgb_inputs(n, nfeat)
    enc = Paillier.encrypt(ctx, embed([g, h], interval=1 << 128, precision=64), precision=0)
    wire = Paillier.serialize(enc, compression=False)
    del enc
    grad_hess = Paillier.ciphertext_from(ctx.to_public(), wire, compression=False)
    data = pd.concat([pd.DataFrame(range(n), columns=['xfl_id']), pd.DataFrame(grad_hess, columns=['xfl_grad_hess']),
                      values], axis=1)
    out = {"dropin_groupby_column_dtype": str(data['xfl_grad_hess'].dtype)}
    cols = list(values.columns)

    def hist(to_numpy):
        res = [data.groupby([c])['xfl_grad_hess'].agg({'count', 'sum'}) for c in cols]
        if to_numpy:
            return [(r['sum'].to_numpy(), r['count'].to_numpy()) for r in res]
        for r in res:
            if isinstance(r['sum'].dtype, PaillierDtype):
                r['sum'].values.is_resident  # noqa: B018 (results computed: the sync below waits for them)
        torch.cuda.synchronize()
        return res
    hist(False)  # first call uploads the column's words once (the later calls read them in HBM)
    torch.cuda.synchronize()
    t0 = time.time()
    res = hist(False)
    out[f"dropin_groupby_100k_x{nfeat}_s"] = time.time() - t0
    t0 = time.time()
    hist(True)
    out[f"dropin_groupby_100k_x{nfeat}_to_numpy_s"] = time.time() - t0
    # check: decrypted bins of 2 features = the exact integer sums of the embedded values
    from xfl_amd.paillier_acceleration import embed as emb
    ints = emb([g, h], interval=1 << 128, precision=64)
    ok = True
    for c in cols[:2]:
        b = values[c].to_numpy()
        got = Paillier.decrypt(ctx, res[cols.index(c)]['sum'].values, out_origin=True)
        want = [sum(ints[b == k].tolist()) for k in res[cols.index(c)].index]
        ok &= [int(v) for v in got] == want
    out["dropin_groupby_bins_exact"] = bool(ok)
    return out


def headline_at_window(nat, L, bits, key_material, win, x, m, ex, st, rnd, N, stream, steps):
    """The headline step (encode + draw + encrypt of N resident float64) on a
    key with `win`-bit tables: the drop-in's starting window is 16
    (context.py WIN_STEPS), so this is what an XFL caller's first calls get."""
    import ctypes
    import torch
    p, q, n, h = key_material
    k = nat.DeviceKey(bits, n, p, q, h, device=torch.cuda.current_device(), win_bits=win)
    ct = torch.empty((N, k.n2w), dtype=torch.int32, device="cuda")
    seed32 = os.urandom(32)

    def step(i):
        nat.check(L.xhe_encode_f64(k.handle, x.data_ptr(), N, 7, 0, 0, m.data_ptr(), ex.data_ptr(), st.data_ptr(),
                                   stream), "encode")
        nat.check(L.xhe_rand(k.handle, seed32, i, N, rnd.data_ptr(), None, stream), "rand")
        nat.check(L.xhe_encrypt(k.handle, m.data_ptr(), rnd.data_ptr(), N, ct.data_ptr(), stream), "encrypt")
    step(0)
    torch.cuda.synchronize()
    L.xhe_profile(1)
    t0 = time.time()
    for i in range(steps):
        step(i + 1)
    torch.cuda.synchronize()
    wall = time.time() - t0
    tot, cnt = ctypes.c_double(), ctypes.c_int64()
    kname = timed_kernel(L, tot, cnt)
    L.xhe_profile(0)
    _, w_pow = algorithmic_macs_per_element(bits, win, k.rand_bits)
    avg = tot.value / max(cnt.value, 1) / 1e3
    rec = {"window_bits": win, "value": N * steps / wall, "unit": "encrypts/s", "ms_per_step": wall / steps * 1e3,
           "kernel": kname, "kernel_avg_ms": avg * 1e3, "frac": N * w_pow / avg / PEAK_MAC_PER_S,
           "table_bytes": nat.table_bytes(bits, win)}
    del k, ct
    return rec


# the fixed-base encryption kernel per key size, as rocprof names it (the
# library's hipEvent scopes carry the same labels): Montgomery digits at
# 2048 (k_djn_pmd) and 3072/4096 (k_djn_pmdx), Montgomery rows through LDS or
# the multi-lane Montgomery kernel otherwise
DJN_KERNELS = ("k_djn_pmd", "k_djn_pmdx", "k_djn_pow_lds", "k_djn_pow")


def timed_kernel(L, tot, cnt):
    """Read the hipEvent totals of whichever DJN kernel ran; returns its name."""
    import ctypes
    from xfl_amd import _native as nat
    for name in DJN_KERNELS:
        nat.check(L.xhe_profile_read(name.encode(), ctypes.byref(tot), ctypes.byref(cnt)))
        if cnt.value:
            return name
    return DJN_KERNELS[-1]


def host_cores():
    """(cores this process may use, cores the machine has): the cgroup CPU
    quota or the affinity mask, whichever is smaller - on the GPU box
    os.cpu_count() shows the whole machine, of which a job gets a share."""
    total = os.cpu_count() or 1
    usable = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else total
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            usable = min(usable, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return usable, total


def cpu_baselines(bits, seconds):
    """cpu_baseline on every usable host core, plus the 1-core leg."""
    usable, total = host_cores()
    rec = cpu_baseline(bits, seconds, usable)
    one = cpu_baseline(bits, max(2.0, seconds / 2), 1)
    rec["machine_cpu_count"] = total
    rec["single_core"] = {"value": one["value"], "unit": one["unit"], "cores": 1, "sample": one["sample"]}
    return rec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--n", type=int, default=1_000_000, help="elements per GPU")
    ap.add_argument("--key-bits", type=int, default=2048)
    ap.add_argument("--win", default="0",
                    help="fixed-base window: w or ws (split, XHE_WIN_SPLIT); 0 = the uniform window with the fewest "
                         "table products whose tables leave 16 GiB of the GPU free (2048 bits: 23, 2 x 96.6 GB, 45 "
                         "products per prime)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-ops", action="store_true", help="skip the secondary-operation rates")
    ap.add_argument("--dist", action="store_true",
                    help="initialise the RCCL process group and gather through it even at --gpus 1 (the N-GPU "
                         "code path - init, async all-gather, barriers, max-over-ranks all-reduce - on one GPU)")
    ap.add_argument("--proxy-world", type=int, default=0,
                    help="with --dist: size the gather target for this many ranks and move the other ranks' share of "
                         "the vector every step too (a one-GPU stand-in for the P-rank job's gather bytes and memory; "
                         "shard.GatherPipeline proxy_world)")
    args = ap.parse_args()

    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        # one process per GPU, started here before anything touches the GPU
        from xfl_amd.shard import spawn_local_ranks
        sys.exit(spawn_local_ranks(args.gpus, [os.path.abspath(__file__)] + sys.argv[1:]))
    if env_world is not None and int(env_world) != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={env_world}; they must agree")

    import torch
    import torch.distributed as dist
    from xfl_amd import _native as nat
    from xfl_amd.shard import GatherPipeline, shard_parity

    world = int(env_world or "1")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    use_dist = world > 1 or args.dist
    if use_dist:
        if env_world is None:  # --dist at one GPU without a launcher: a group of one rank
            from xfl_amd.shard import free_port
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", str(free_port()))
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", local))

    bits = args.key_bits
    p, q, n, h = make_key(bits, seed=2024)
    args.win = nat.parse_win(args.win)
    if args.win == 0:
        args.win = pick_window(bits, torch.cuda.mem_get_info(local)[0])
    t_key = time.time()
    dk = nat.DeviceKey(bits, n, p, q, h, device=local, win_bits=args.win)
    torch.cuda.synchronize()
    t_key = time.time() - t_key
    L = nat.lib()

    N = args.n
    rng = np.random.default_rng(0 + rank)
    x = torch.from_numpy(rng.standard_normal(N)).to("cuda")
    m = torch.empty((N, dk.nw), dtype=torch.int32, device="cuda")
    ex = torch.empty(N, dtype=torch.int32, device="cuda")
    st = torch.empty(N, dtype=torch.int32, device="cuda")
    rnd = torch.empty((N, dk.rand_words), dtype=torch.int32, device="cuda")
    seed32 = os.urandom(32)
    stream = torch.cuda.current_stream().cuda_stream

    def encrypt_shard(i, ct):
        nat.check(L.xhe_encode_f64(dk.handle, x.data_ptr(), N, 7, 0, 0, m.data_ptr(), ex.data_ptr(),
                                   st.data_ptr(), stream), "encode")
        nat.check(L.xhe_rand(dk.handle, seed32, i, N, rnd.data_ptr(), None, stream), "rand")
        nat.check(L.xhe_encrypt(dk.handle, m.data_ptr(), rnd.data_ptr(), N, ct.data_ptr(), stream), "encrypt")

    pipe = GatherPipeline(encrypt_shard, N, dk.n2w, world=world, rank=rank, device="cuda", collective=use_dist,
                          proxy_world=args.proxy_world or None)
    last = 1_000_000 + max(args.warmup, 1) - 1  # the parity check below needs one finished step
    for i in range(1_000_000, last + 1):
        pipe.step(i)
    pipe.drain()
    torch.cuda.synchronize()
    # parity check of this rank's output (not timed): 4,096 elements spread
    # over the shard against the reference's encryption on the same draws -
    # the oracle's encode (encoder.py:29-54) and the GMP port's DJN-CRT
    # encryption (oracle/gmp_baseline.c, pinned to the golden ciphertexts);
    # the pure-Python oracle on 4 of them when libgmp is not loadable
    from oracle import bench_cpu
    from oracle import paillier_oracle as O
    okey = O.derive_private(p, q, h)
    xs = x.cpu().numpy()
    rnd_h = rnd.cpu().numpy().view(np.uint32)
    idx = np.unique(np.concatenate([[0, 1, N // 2, N - 1], np.random.default_rng(7).integers(0, N, 4092)]))
    ms = [O.encode_element(okey, float(xs[i]), 7)[0] for i in idx]
    try:
        want = bench_cpu.gmp_encrypt_batch(okey, nat.ints_to_words(ms, dk.nw), rnd_h[idx], threads=host_cores()[0])
        want = dict(zip(idx.tolist(), nat.words_to_ints(want)))
    except RuntimeError:
        idx = idx[[0, 1, -2, -1]]
        want = {int(i): O.encrypt_m(okey, O.encode_element(okey, float(xs[i]), 7)[0], nat.words_to_ints(rnd_h[i]))
                for i in idx}
    parity_n = len(idx)
    parity_ok = shard_parity(pipe.shard(last), pipe.vector(last) if use_dist else None, rank, [int(i) for i in idx],
                             want.__getitem__)

    free_after = int(torch.cuda.mem_get_info(local)[0])
    L.xhe_profile(1)
    if use_dist:
        dist.barrier()
    torch.cuda.synchronize()
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.time()
    ev0.record()
    for i in range(args.steps):
        ct = pipe.step(i)
    pipe.drain()
    ev1.record()
    torch.cuda.synchronize()
    if use_dist:
        dist.barrier()
    wall = time.time() - t0
    ms_total = ev0.elapsed_time(ev1)
    import ctypes
    tot = ctypes.c_double()
    cnt = ctypes.c_int64()
    kname = timed_kernel(L, tot, cnt)
    L.xhe_profile(0)
    elapsed = max(wall, ms_total / 1e3)
    if use_dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        ok = torch.tensor([1 if parity_ok else 0], dtype=torch.int32, device="cuda")
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        parity_ok = bool(ok.item())

    value = world * N * args.steps / elapsed
    if rank == 0:
        w_elem, w_pow = algorithmic_macs_per_element(bits, args.win, dk.rand_bits)
        pow_avg_s = (tot.value / max(cnt.value, 1)) / 1e3
        achieved = N * w_pow / pow_avg_s / 1e12  # N elements x 2 primes per launch
        traffic, traffic_src, pmc = pmc_traffic(args.win, N, kname) if bits == 2048 else (None, None, None)
        rec = {
            "metric": "2048-bit Paillier encrypts/s (device-resident)" if bits == 2048 else f"{bits}-bit Paillier encrypts/s (device-resident)",
            "value": value, "unit": "encrypts/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u32", "data": "synthetic",
            "config": {"workload": f"DJN private-key (CRT) encrypt, obfuscated, precision 7, {N} float64 "
                                   f"plaintexts/GPU resident in HBM" + (", + RCCL all-gather" if use_dist else ""),
                       "key_bits": bits, "elements_per_gpu": N, "fixed_base_window_bits": args.win & 0xFF,
                       "fixed_base_window_split": bool(args.win & nat.XHE_WIN_SPLIT),
                       "parallelism": f"shard{world}" + ("+rccl" if use_dist else "")},
            "roofline": {"bound": "valu-int", "achieved": achieved, "peak": PEAK_MAC_PER_S / 1e12,
                         "unit": "TMAC/s", "frac": achieved * 1e12 / PEAK_MAC_PER_S, "traffic": traffic,
                         "traffic_source": traffic_src, "kernel": kname, "kernel_avg_ms": pow_avg_s * 1e3,
                         "alg_macs_per_element": w_pow,
                         "alg_table_bytes_per_launch": N * 2 * nat.win_layout(dk.rand_bits, args.win)[0] * TABLE_ROW_BYTES[bits]},
            "parity_sample_ok": parity_ok,
            "parity_sample_n": parity_n,
            "key_setup_s": t_key,
            "hbm_free_after_setup_bytes": free_after,
        }
        if pipe.proxy:
            rec["config"]["proxy_world"] = pipe.proxy
            rec["config"]["proxy_gather_bytes_per_step"] = (pipe.proxy - world) * N * dk.n2w * 4
            rec["config"]["gather_target_bytes"] = sum(g.numel() * 4 for g in pipe.gathered)
        hm = issued_mads(bits, (p, q, n, h), args.win).get("headline")
        if hm:  # the kernel's own schedule (digit products), not the 8(d) model
            rec["roofline"]["issued_mads_per_element"] = hm
            rec["roofline"]["issued_mad_frac"] = N * hm / pow_avg_s / PEAK_MAC_PER_S
        if pmc and pmc.get("clock_ghz"):
            # the counter pass's clock under this load (SQ_BUSY_CYCLES) and VALU
            # busy: `peak` is the 2.4 GHz figure, the kernel runs below it
            rec["roofline"].update({"pmc_clock_ghz": float(pmc["clock_ghz"]),
                                    "pmc_valu_busy_frac": pmc.get("valu_busy_frac")})
        rec["config"]["table_bytes"] = nat.table_bytes(bits, args.win)
        if not args.no_ops and (args.win & 0xFF) != 16:
            rec["headline_dropin_window"] = headline_at_window(nat, L, bits, (p, q, n, h), 16, x, m, ex, st, rnd, N,
                                                               stream, args.steps)
        if not args.no_ops:
            rec["ops"] = measure_ops(nat, L, dk, x, m, ex, ct, rnd, N, stream, (p, q, n, h))
            # the drop-in with its own context and window policy: the bench
            # key's tables (193 GB at window 23) are released first
            dev, xh = dk.device, x[:min(N, 1 << 20)].cpu().numpy()
            del pipe, encrypt_shard, dk
            import gc
            gc.collect()
            torch.cuda.empty_cache()
            rec["ops"].update(measure_dropin(nat, dev, bits, xh, (p, q, n, h)))
            clock = float(pmc["clock_ghz"]) if pmc and pmc.get("clock_ghz") else None
            rec["ops"]["issued"] = issued_fractions(rec["ops"], bits, (p, q, n, h), args.win, N / pow_avg_s, clock)
        if not args.no_cpu_baseline:
            rec["cpu_baseline"] = cpu_baselines(bits, args.cpu_seconds)
        print(json.dumps(rec), flush=True)
    if use_dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
