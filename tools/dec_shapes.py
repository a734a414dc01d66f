"""Decrypt latency/throughput per batch size for one exponentiation shape
(XHE_DEC_TPI = 1, 4 or 16 pins it; unset = the library's choice by size).
Device-resident ciphertexts, hipEvent-free wall time of xhe_decrypt +
synchronize, median of repeats. Prints one JSON line.

    XHE_DEC_TPI=16 python tools/dec_shapes.py
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
    sizes = [int(a) for a in sys.argv[1:]] or [1, 15, 64, 256, 1024, 2048, 4096, 16384, 65536]
    N = max(sizes)
    rng = np.random.default_rng(1)
    c = torch.from_numpy(rng.integers(0, 2 ** 32, (N, dk.n2w), dtype=np.uint64).astype(np.uint32).view(np.int32))
    c[:, -1] = c[:, -1] & 0x0FFFFFFF  # below n^2's top word range
    c = c.cuda()
    m = torch.empty((N, dk.nw), dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    out = {"tpi": os.environ.get("XHE_DEC_TPI", "auto")}
    for k in sizes:
        ts = []
        for _ in range(5):
            torch.cuda.synchronize()
            t = time.perf_counter()
            nat.check(L.xhe_decrypt(dk.handle, c.data_ptr(), k, m.data_ptr(), s))
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t)
        ts.sort()
        out[str(k)] = {"ms": round(ts[2] * 1e3, 3), "per_s": round(k / ts[2])}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
