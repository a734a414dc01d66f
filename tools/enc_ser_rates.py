"""The label trainer's Paillier.encrypt -> Paillier.serialize(compression=True)
on 1 M float32 residuals through the drop-in (device-resident result,
pipelined serialize), and the encrypt alone, at the context's starting window
16: one JSON line (median of 5). $XHE_ENC_SUB sets the rows per encryption
launch (A/B).
    python tools/enc_ser_rates.py [n]
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
    from xfl_amd.paillier import Paillier, PaillierContext
    from xfl_amd.paillier import wire
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    p, q, nn, h = make_key(2048, seed=2024)
    ctx = PaillierContext().init(p, q, djn_h_pow_n=h)
    x = np.random.default_rng(1).standard_normal(n).astype(np.float32)
    out = {"n": n, "enc_sub": wire.ENC_SUB}

    def timed(f, reps=5):
        ts = []
        for _ in range(reps):
            ctx._volume = 0  # stay at window 16
            torch.cuda.synchronize()
            t = time.perf_counter()
            f()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t)
        return sorted(ts)[reps // 2]
    keep = {}

    def enc():
        keep.pop(0, None)
        keep[0] = Paillier.encrypt(ctx, x, precision=7)

    def enc_ser():
        keep.pop(1, None)
        keep[1] = Paillier.serialize(Paillier.encrypt(ctx, x, precision=7), compression=True)
    enc()
    enc_ser()
    out["encrypt_per_s"] = n / timed(enc)
    keep.clear()
    out["encrypt_serialize_zstd_per_s"] = n / timed(enc_ser)
    out["window"] = ctx._dev[torch.cuda.current_device()].win_bits
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
