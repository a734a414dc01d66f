"""Cycle budget of one k_dec_rns product (a probe build: python -m xfl_amd.build
--out xfl_amd/lib/probe/libxhe.so -D XHE_RNS_PROBE=1 -D XHE_ONLY_2048, run with
XHE_LIB pointing at it). Decrypts a small batch through the RNS shape, then
reads block (0, 0)'s per-role phase clocks (rns_dev.hpp) and prints one JSON
line: clocks per product for phase 1 (products + first barrier), phase 2 (B'
extension + second barrier), phase 3 (B extension), per role, and the shader
clock rate from the 100 MHz real-time counter.
    XHE_LIB=xfl_amd/lib/probe/libxhe.so python tools/rns_probe.py [batch]
"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    from bench import make_key
    from xfl_amd import _native as nat
    n_el = int(sys.argv[1]) if len(sys.argv) > 1 else 15
    p, q, n, h = make_key(2048, seed=2024)
    dk = nat.DeviceKey(2048, n, p, q, h, win_bits=16)
    L = nat.lib()
    rng = np.random.default_rng(1)
    c = torch.from_numpy(rng.integers(0, 2 ** 32, (n_el, dk.n2w), dtype=np.uint64).astype(np.uint32).view(np.int32))
    c[:, -1] = c[:, -1] & 0x0FFFFFFF
    c = c.cuda()
    m = torch.empty((n_el, dk.nw), dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    out = {}
    for rep in range(3):
        nat.check(L.xhe_decrypt(dk.handle, c.data_ptr(), n_el, m.data_ptr(), s), "decrypt")
        torch.cuda.synchronize()
        buf = (ctypes.c_ulonglong * 16)()
        fn = L.xhe_rns_probe_read
        fn.argtypes = [ctypes.c_void_p]
        nat.check(fn(buf), "probe")
        v = list(buf)
        ghz = v[8] / (v[9] / 100e6) / 1e9 if v[9] else None
        roles = {}
        for name, o in (("B", 0), ("B2", 4)):
            cnt = max(v[o + 3], 1)
            roles[name] = {"phase1": v[o] / cnt, "phase2": v[o + 1] / cnt, "phase3": v[o + 2] / cnt,
                           "products": v[o + 3]}
        out = {"batch": n_el, "kernel_clocks": v[8], "kernel_us": v[9] / 100.0, "clock_ghz": ghz,
               "clocks_per_product": (v[0] + v[1] + v[2]) / max(v[3], 1), "roles": roles}
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
