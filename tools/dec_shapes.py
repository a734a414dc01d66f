"""Decrypt (or, with --enc, DJN private encrypt) latency/throughput per batch
size for one lane shape: XHE_DEC_TPI = 1, 4 or 16 pins the decrypt shape,
XHE_ENC_TPI = 16 or 0 the encrypt one; unset = the library's choice by size.
Device-resident operands, wall time of the call + synchronize, median of 5.
Prints one JSON line.

    XHE_DEC_TPI=16 python tools/dec_shapes.py [sizes...]
    XHE_ENC_TPI=0 python tools/dec_shapes.py --enc [sizes...]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    from bench import make_key
    from xfl_amd import _native as nat
    p, q, n, h = make_key(2048, seed=2024)
    dk = nat.DeviceKey(2048, n, p, q, h, win_bits=16)
    L = nat.lib()
    enc = "--enc" in sys.argv
    sizes = [int(a) for a in sys.argv[1:] if a != "--enc"] or [1, 15, 64, 256, 1024, 2048, 4096, 16384, 65536]
    N = max(sizes)
    rng = np.random.default_rng(1)
    c = torch.from_numpy(rng.integers(0, 2 ** 32, (N, dk.n2w), dtype=np.uint64).astype(np.uint32).view(np.int32))
    c[:, -1] = c[:, -1] & 0x0FFFFFFF  # below n^2's top word range
    c = c.cuda()
    m = torch.empty((N, dk.nw), dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    out = {"op": "encrypt" if enc else "decrypt",
           "tpi": os.environ.get("XHE_ENC_TPI" if enc else "XHE_DEC_TPI", "auto")}
    if enc:
        m.random_(0, 1 << 30)
        m[:, -1] = 0
        r = torch.randint(0, 1 << 30, (N, dk.rand_words), dtype=torch.int32, device="cuda")
    for k in sizes:
        ts = []
        for _ in range(5):
            torch.cuda.synchronize()
            t = time.perf_counter()
            if enc:
                nat.check(L.xhe_encrypt(dk.handle, m.data_ptr(), r.data_ptr(), k, c.data_ptr(), s))
            else:
                nat.check(L.xhe_decrypt(dk.handle, c.data_ptr(), k, m.data_ptr(), s))
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t)
        ts.sort()
        out[str(k)] = {"ms": round(ts[2] * 1e3, 3), "per_s": round(k / ts[2])}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
