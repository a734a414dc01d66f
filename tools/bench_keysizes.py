"""Per-key-size rates on one GPU (2048/3072/4096/8192-bit DJN private keys):
DJN-CRT encrypt (encode + draw + encrypt, precision 7, obfuscated) and CRT
decrypt of the same ciphertexts, with the round trip checked bit-exactly.

Keys are the reference-generated fixture keys (tests/golden/paillier_K_djn.json)
so no host key generation runs here (pure-Python keygen of an 8192-bit DJN
key takes minutes).

    python tools/bench_keysizes.py [--bits 2048,3072,4096,8192] > profiles/r1/keysizes.jsonl
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

from tools.bench_configs import _encrypt_f64, _sync, _timed  # noqa: E402

# elements per timed call: enough lanes to fill the chip in the batch shapes
N_BY_BITS = {2048: 1_000_000, 3072: 500_000, 4096: 262_144, 8192: 65_536}
# --win 0: each size at the widest window whose packed tables leave 16 GiB of
# HBM free (bench.pick_window), as bench.py --key-bits K picks it


def run(bits, steps, win):
    import torch
    from tests.conftest import hx, load_fixture
    from xfl_amd import _native as nat
    L = nat.lib()
    k = load_fixture(f"paillier_{bits}_djn.json")["key"]
    p, q, h = hx(k["p"]), hx(k["q"]), hx(k["h_pow_n"])
    if not win:
        from bench import pick_window
        win = pick_window(bits, torch.cuda.mem_get_info(0)[0])
    t0 = time.time()
    dk = nat.DeviceKey(bits, p * q, p, q, h, device=0, win_bits=win)
    _sync()
    tk = time.time() - t0
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
    td = _timed(lambda: nat.check(L.xhe_decrypt(dk.handle, ct.data_ptr(), N, m2.data_ptr(), s), "decrypt"), steps)
    _sync()
    # SURVEY 8(d) model: 2 nwin table products of s = K/32 limbs at 2s^2+s
    # MACs (bench.py's roofline.achieved), over the measured v_mad peak
    s_ = bits // 32
    macs = 2 * nat.win_layout(dk.rand_bits, win)[0] * (2 * s_ * s_ + s_)
    out = {"key_bits": bits, "elements": N, "fixed_base_window": nat.win_spec(win),
           "encrypts_per_s": N / te, "decrypts_per_s": N / td,
           "alg_macs_per_encrypt": macs, "encrypt_tmac_per_s": N / te * macs / 1e12,
           "encrypt_roofline_frac": N / te * macs / 39.3216e12,
           "roundtrip_bit_exact": bool(torch.equal(m, m2)), "key_setup_s": tk}
    del dk
    torch.cuda.empty_cache()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bits", default="2048,3072,4096,8192")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--win", default="0", help="window for every size (w or ws = split); 0 = fewest products that fit")
    a = ap.parse_args()
    for b in [int(v) for v in a.bits.split(",")]:
        from xfl_amd._native import parse_win
        print(json.dumps(run(b, a.steps, parse_win(a.win))), flush=True)


if __name__ == "__main__":
    main()
