"""Rates of the operations round 4 moved to Montgomery digits, for same-box A/B
runs (the $XHE_* switches select the old kernels; they are read once per
process, so each side of an A/B is its own process):

  private non-DJN encrypt, 2048 bits    $XHE_NODJN_PMD=0 -> k_nodjn_crt (Montgomery)
  public DJN encrypt, 2048 bits (w16)   $XHE_NDIG_PUB=0  -> k_djn_pub (Montgomery n^2 tables)
  decrypt, 3072 / 4096 bits (batches)   $XHE_DEC_PMDX=0  -> k_dec_pow 4-lane (Montgomery)
  ciphertext add / 1 M-element sum      (no switch: the round-4 product counts)
  LR-shaped latency ops (B = 64, D = 15) $XHE_MEXP_WAVE=0 / $XHE_ADD_WAVE=0 -> the 16-lane
                                        Horner / aligned add instead of one 16-wave block each

Each rate comes with a checksum of the outputs so the two sides can be
compared for equality.

    python tools/rates_r4.py [--only nodjn,pub,dec3072,dec4096,add,sum,pubnodjn,lr,matvec] > out.jsonl
"""
import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def _timed(fn, reps):
    import torch
    fn()
    torch.cuda.synchronize()
    t0 = time.time()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.time() - t0) / reps


def _sum(t):
    return hashlib.sha1(t.cpu().numpy().tobytes()).hexdigest()[:16]


def _rand_words(rng, n, words, top_bits=None):
    import torch
    w = rng.integers(0, 1 << 32, size=(n, words), dtype=np.uint64).astype(np.uint32)
    if top_bits is not None:
        w[:, -1] &= np.uint32((1 << top_bits) - 1)
    return torch.from_numpy(w.view(np.int32)).cuda()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="nodjn,pub,dec3072,dec4096,add,sum,pubnodjn,lr,matvec")
    args = ap.parse_args()
    only = set(args.only.split(","))
    import torch
    from tests.conftest import hx, load_fixture
    from xfl_amd import _native as nat
    L = nat.lib()
    s = torch.cuda.current_stream().cuda_stream
    env = {k: v for k, v in os.environ.items() if k.startswith("XHE_")}
    rng = np.random.default_rng(1)

    def out(rec):
        rec["env"] = env
        print(json.dumps(rec), flush=True)

    k = load_fixture("paillier_2048_djn.json")["key"]
    p, q, h = hx(k["p"]), hx(k["q"]), hx(k["h_pow_n"])
    n = p * q
    if "nodjn" in only:
        dk = nat.DeviceKey(2048, n, p, q, None, device=0)
        N = 65536
        m = _rand_words(rng, N, dk.nw, 30)
        r = _rand_words(rng, N, dk.rand_words, 30)
        ct = torch.empty((N, dk.n2w), dtype=torch.int32, device="cuda")
        t = _timed(lambda: nat.check(L.xhe_encrypt(dk.handle, m.data_ptr(), r.data_ptr(), N, ct.data_ptr(), s)), 3)
        out({"op": "encrypt_private_nodjn_2048", "n": N, "per_s": N / t, "ms": t * 1e3, "sum": _sum(ct)})
        del dk
    if "pub" in only:
        dk = nat.DeviceKey(2048, n, None, None, h, device=0, win_bits=16)
        N = 1 << 20
        m = _rand_words(rng, N, dk.nw, 30)
        r = _rand_words(rng, N, dk.rand_words)
        ct = torch.empty((N, dk.n2w), dtype=torch.int32, device="cuda")
        t = _timed(lambda: nat.check(L.xhe_encrypt(dk.handle, m.data_ptr(), r.data_ptr(), N, ct.data_ptr(), s)), 3)
        out({"op": "encrypt_public_djn_2048_w16", "n": N, "per_s": N / t, "ms": t * 1e3, "sum": _sum(ct)})
        if "add" in only or "sum" in only:
            N2 = 1 << 20
            a, b = ct[:N2], torch.roll(ct, 1, 0)[:N2].contiguous()
            o = torch.empty_like(a)
            if "add" in only:
                t = _timed(lambda: nat.check(L.xhe_mulmod(dk.handle, a.data_ptr(), None, b.data_ptr(), None, N2, 0,
                                                          o.data_ptr(), None, s)), 5)
                out({"op": "add_2048", "n": N2, "per_s": N2 / t, "ms": t * 1e3, "sum": _sum(o)})
            if "sum" in only:
                import ctypes
                seg = np.array([0, N2], dtype=np.int64)
                o1 = torch.empty((1, dk.n2w), dtype=torch.int32, device="cuda")
                t = _timed(lambda: nat.check(L.xhe_segprod(dk.handle, a.data_ptr(), None, 0, N2,
                                                           seg.ctypes.data_as(ctypes.c_void_p), 1, o1.data_ptr(), s)), 3)
                out({"op": "sum_2048", "n": N2, "per_s": N2 / t, "ms": t * 1e3, "sum": _sum(o1)})
                nb = 256
                segh = (np.arange(nb + 1, dtype=np.int64) * (100_000 // nb))
                segh[-1] = 100_000
                oh = torch.empty((nb, dk.n2w), dtype=torch.int32, device="cuda")
                t = _timed(lambda: nat.check(L.xhe_segprod(dk.handle, a.data_ptr(), None, 0, 100_000,
                                                           segh.ctypes.data_as(ctypes.c_void_p), nb, oh.data_ptr(), s)), 3)
                out({"op": "hist_256x100k_2048", "n": 100_000, "ms": t * 1e3, "sum": _sum(oh)})
        del dk
    if "pubnodjn" in only or "matvec" in only or "lr" in only:
        dk = nat.DeviceKey(2048, n, None, None, None, device=0)
        if "pubnodjn" in only:
            N = 65536
            m = _rand_words(rng, N, dk.nw, 30)
            r = _rand_words(rng, N, dk.rand_words, 30)
            ct = torch.empty((N, dk.n2w), dtype=torch.int32, device="cuda")
            t = _timed(lambda: nat.check(L.xhe_encrypt(dk.handle, m.data_ptr(), r.data_ptr(), N, ct.data_ptr(), s)), 2)
            out({"op": "encrypt_public_nodjn_2048", "n": N, "per_s": N / t, "ms": t * 1e3, "sum": _sum(ct)})
        if "lr" in only:
            # the LR step's latency-bound shapes (B = 64, D = 15): aligned add of
            # 15 ciphertexts with a 50-step gap (+ noise), mat-vec 64 x 15 at 70 bits
            Ns = 15
            a_ = _rand_words(rng, Ns, dk.n2w, 30)
            b_ = _rand_words(rng, Ns, dk.n2w, 30)
            ea_ = torch.full((Ns,), -60, dtype=torch.int32, device="cuda")
            eb_ = torch.full((Ns,), -10, dtype=torch.int32, device="cuda")
            o_ = torch.empty_like(a_)
            eo_ = torch.empty_like(ea_)
            t = _timed(lambda: nat.check(L.xhe_mulmod(dk.handle, a_.data_ptr(), ea_.data_ptr(), b_.data_ptr(),
                                                      eb_.data_ptr(), Ns, 50, o_.data_ptr(), eo_.data_ptr(), s)), 5)
            out({"op": "add_aligned_15_d50", "ms": t * 1e3, "sum": _sum(o_)})
            B, D, kb = 64, 15, 70
            bases = _rand_words(rng, B, dk.n2w, 30)
            idx = torch.from_numpy(np.tile(np.arange(B, dtype=np.int32), (D, 1))).cuda()
            kx = _rand_words(rng, D * B, 3, kb - 64)
            mv = torch.empty((D, dk.n2w), dtype=torch.int32, device="cuda")
            t = _timed(lambda: nat.check(L.xhe_multiexp(dk.handle, bases.data_ptr(), B, idx.data_ptr(), kx.data_ptr(),
                                                        3, kb, D, B, 0, mv.data_ptr(), s)), 5)
            out({"op": "matvec_64x15_70bit", "ms": t * 1e3, "sum": _sum(mv)})
        if "matvec" in only:
            # the bench's mat-vec: 2048 ciphertext bases x 15 columns, 53-bit exponents
            B, D, kb = 2048, 15, 53
            bases = _rand_words(rng, B, dk.n2w, 30)
            idx = torch.from_numpy(np.tile(np.arange(B, dtype=np.int32), (D, 1))).cuda()
            kx = _rand_words(rng, D * B, 2, kb - 32)
            mv = torch.empty((D, dk.n2w), dtype=torch.int32, device="cuda")
            t = _timed(lambda: nat.check(L.xhe_multiexp(dk.handle, bases.data_ptr(), B, idx.data_ptr(), kx.data_ptr(),
                                                        2, kb, D, B, 0, mv.data_ptr(), s)), 3)
            out({"op": "matvec_2048x15", "ms": t * 1e3, "terms_per_s": B * D / t, "sum": _sum(mv)})
        del dk
    for bits in (3072, 4096):
        if f"dec{bits}" not in only:
            continue
        kk = load_fixture(f"paillier_{bits}_djn.json")["key"]
        p, q, h = hx(kk["p"]), hx(kk["q"]), hx(kk["h_pow_n"])
        dk = nat.DeviceKey(bits, p * q, p, q, h, device=0, win_bits=12)
        N = 500_000 if bits == 3072 else 262_144
        m = _rand_words(rng, N, dk.nw, 30)
        r = _rand_words(rng, N, dk.rand_words, 30)
        ct = torch.empty((N, dk.n2w), dtype=torch.int32, device="cuda")
        nat.check(L.xhe_encrypt(dk.handle, m.data_ptr(), r.data_ptr(), N, ct.data_ptr(), s))
        mo = torch.empty((N, dk.nw), dtype=torch.int32, device="cuda")
        t = _timed(lambda: nat.check(L.xhe_decrypt(dk.handle, ct.data_ptr(), N, mo.data_ptr(), s)), 2)
        out({"op": f"decrypt_{bits}", "n": N, "per_s": N / t, "ms": t * 1e3, "roundtrip": bool(torch.equal(mo, m))})
        del dk


if __name__ == "__main__":
    main()
