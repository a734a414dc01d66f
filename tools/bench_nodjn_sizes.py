"""Private-key non-DJN encryption (r^ep mod p^2 / r^eq mod q^2 + CRT,
paillier.py:214-230) per key size on one GPU, round trip checked: exposes
limb shapes that spill in the variable-base exponentiation.

    python tools/bench_nodjn_sizes.py [--bits 2048,3072,4096]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from tools.bench_configs import _encrypt_f64, _sync, _timed  # noqa: E402

N_BY_BITS = {2048: 131072, 3072: 65536, 4096: 32768, 8192: 4096}


def run(bits, steps):
    import torch
    from tests.conftest import hx, load_fixture
    from xfl_amd import _native as nat
    L = nat.lib()
    k = load_fixture(f"paillier_{bits}_djn.json")["key"]
    p, q = hx(k["p"]), hx(k["q"])
    dk = nat.DeviceKey(bits, p * q, p, q, None, device=0)
    N = N_BY_BITS[bits]
    x = torch.from_numpy(np.random.default_rng(2).standard_normal(N)).cuda()
    m = torch.empty((N, dk.nw), dtype=torch.int32, device="cuda")
    m2 = torch.empty_like(m)
    ex = torch.empty(N, dtype=torch.int32, device="cuda")
    st = torch.empty_like(ex)
    rnd = torch.empty((N, dk.rand_words), dtype=torch.int32, device="cuda")
    ct = torch.empty((N, dk.n2w), dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    te = _timed(lambda: _encrypt_f64(nat, L, dk, x, 7, m, ex, st, rnd, ct, 1, s), steps)
    nat.check(L.xhe_decrypt(dk.handle, ct.data_ptr(), N, m2.data_ptr(), s), "decrypt")
    _sync()
    return {"key_bits": bits, "mode": "private non-DJN", "elements": N, "encrypts_per_s": N / te,
            "roundtrip_bit_exact": bool(torch.equal(m, m2))}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bits", default="2048,3072,4096")
    ap.add_argument("--steps", type=int, default=2)
    a = ap.parse_args()
    for b in [int(v) for v in a.bits.split(",")]:
        print(json.dumps(run(b, a.steps)), flush=True)


if __name__ == "__main__":
    main()
