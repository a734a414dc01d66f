"""Same-box A/B of the mod-n^2 exponentiations: public non-DJN encryption
(r^n, paillier.py:228-230) and the scalar power c^k of the batch shape
(53-bit k, paillier.py:156-187), Montgomery digits (default) vs the Montgomery
kernels ($XHE_NDIG=0). Each setting runs in its own process (the switch is
read once); prints one JSON line per setting.

    python tools/ab_ndig.py [--n 65536]
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(n):
    sys.path.insert(0, ROOT)
    import numpy as np
    import torch
    from bench import make_key
    from xfl_amd import _native as nat
    p, q, nn, h = make_key(2048, seed=2024)
    L = nat.lib()
    s = torch.cuda.current_stream().cuda_stream
    pub = nat.DeviceKey(2048, nn, None, None, None, device=0)
    rng = np.random.default_rng(1)
    m = torch.from_numpy(rng.integers(0, 2 ** 31, (n, pub.nw), dtype=np.int64).astype(np.int32)).cuda()
    m[:, -1] = 0
    r = torch.empty((n, pub.rand_words), dtype=torch.int32, device="cuda")
    nat.check(L.xhe_rand(pub.handle, b"\x02" * 32, 3, n, r.data_ptr(), None, s), "rand")
    ct = torch.empty((n, pub.n2w), dtype=torch.int32, device="cuda")

    def timed(fn, reps):
        fn()
        torch.cuda.synchronize()
        t0 = time.time()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        return (time.time() - t0) / reps
    t = timed(lambda: nat.check(L.xhe_encrypt(pub.handle, m.data_ptr(), r.data_ptr(), n, ct.data_ptr(), s), "enc"), 2)
    out = {"ndig": os.environ.get("XHE_NDIG", "1"), "n": n, "encrypt_public_nodjn_per_s": n / t}
    k = torch.from_numpy(rng.integers(0, 2 ** 31, (n, 2), dtype=np.int64).astype(np.int32)).cuda()
    k[:, 1] &= (1 << 21) - 1
    k[:, 1] |= 1 << 20
    c2 = torch.empty_like(ct)
    t = timed(lambda: nat.check(L.xhe_powmod(pub.handle, ct.data_ptr(), k.data_ptr(), 2, 53, n, c2.data_ptr(), s),
                                "powmod"), 3)
    out["scalar_mul_53bit_per_s"] = n / t
    # the two settings must agree bit for bit: a checksum of the outputs
    out["checksum"] = int(torch.sum(c2.to(torch.int64) * torch.arange(1, c2.shape[1] + 1, device="cuda")).item())
    out["checksum_enc"] = int(torch.sum(ct.to(torch.int64) * torch.arange(1, ct.shape[1] + 1, device="cuda")).item())
    print(json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--child", action="store_true")
    a = ap.parse_args()
    if a.child:
        child(a.n)
        return
    for v in ("1", "0", "1"):
        env = dict(os.environ, XHE_NDIG=v)
        subprocess.run([sys.executable, os.path.abspath(__file__), "--child", "--n", str(a.n)], env=env, check=True)


if __name__ == "__main__":
    main()
