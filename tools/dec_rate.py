"""Decrypt and non-DJN encrypt rates of one library build (A/B of kernel
variants through $XHE_LIB): 2048-bit fixture key, device-resident buffers.

    XHE_LIB=xfl_amd/lib/libxhe_dev.so python tools/dec_rate.py [--n 524288]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def main():
    import torch
    from tests.conftest import hx, load_fixture
    from xfl_amd import _native as nat
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=524288)
    ap.add_argument("--steps", type=int, default=3)
    a = ap.parse_args()
    L = nat.lib()
    k = load_fixture("paillier_2048_djn.json")["key"]
    p, q, h = hx(k["p"]), hx(k["q"]), hx(k["h_pow_n"])
    n = p * q
    N = a.n
    s = torch.cuda.current_stream().cuda_stream
    rng = np.random.default_rng(5)
    out = {"lib": os.path.basename(os.environ.get("XHE_LIB", "libxhe.so")), "n": N}

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        t = time.time()
        for _ in range(a.steps):
            fn()
        torch.cuda.synchronize()
        return (time.time() - t) / a.steps

    dk = nat.DeviceKey(2048, n, p, q, h, device=0, win_bits=16)
    mw = torch.from_numpy(rng.integers(0, 1 << 32, (N, dk.nw), dtype=np.uint32).view(np.int32)).cuda()
    mw[:, -1] &= 0x3FFFFFFF  # m < n
    rnd = torch.empty((N, dk.rand_words), dtype=torch.int32, device="cuda")
    ct = torch.empty((N, dk.n2w), dtype=torch.int32, device="cuda")
    m2 = torch.empty_like(mw)
    nat.check(L.xhe_rand(dk.handle, b"\x03" * 32, 1, N, rnd.data_ptr(), None, s), "rand")
    nat.check(L.xhe_encrypt(dk.handle, mw.data_ptr(), rnd.data_ptr(), N, ct.data_ptr(), s), "encrypt")
    td = timed(lambda: nat.check(L.xhe_decrypt(dk.handle, ct.data_ptr(), N, m2.data_ptr(), s), "decrypt"))
    out["decrypt_per_s"] = N / td
    out["decrypt_bit_exact"] = bool(torch.equal(mw, m2))
    # private non-DJN (r^ep mod p^2 CRT) and public non-DJN (r^n mod n^2)
    nk = nat.DeviceKey(2048, n, p, q, None, device=0)
    r2 = torch.empty((N // 8, nk.rand_words), dtype=torch.int32, device="cuda")
    c2 = torch.empty((N // 8, nk.n2w), dtype=torch.int32, device="cuda")
    nat.check(L.xhe_rand(nk.handle, b"\x04" * 32, 1, N // 8, r2.data_ptr(), None, s), "rand")
    te = timed(lambda: nat.check(L.xhe_encrypt(nk.handle, mw.data_ptr(), r2.data_ptr(), N // 8, c2.data_ptr(), s),
                                 "encrypt"))
    out["encrypt_private_nodjn_per_s"] = (N // 8) / te
    d2 = torch.empty((N // 8, nk.nw), dtype=torch.int32, device="cuda")
    nat.check(L.xhe_decrypt(nk.handle, c2.data_ptr(), N // 8, d2.data_ptr(), s), "decrypt")
    torch.cuda.synchronize()
    out["nodjn_roundtrip_bit_exact"] = bool(torch.equal(mw[:N // 8], d2))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
