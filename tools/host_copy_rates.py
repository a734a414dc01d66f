"""Host-buffer encrypt rates (PCIe-inclusive) for the copy-out path of
xhe_encrypt_f64_host / xhe_encrypt_words_host, on one GPU:

    python tools/host_copy_rates.py [--n 1000000] [--win 20]

Times 1 M float64 -> ciphertext words into (a) a fresh np.empty per call,
(b) a fresh nat.empty (hugepage-advised, pre-faulted) per call, (c) one
reused buffer, plus the drop-in Paillier.encrypt and encrypt + serialize,
and checks the host result bit-exactly against the device-resident call.
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--win", type=int, default=20)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import torch
    from bench import make_key
    from xfl_amd import _native as nat
    from xfl_amd.paillier import Paillier, PaillierContext

    p, q, n, h = make_key(2048, seed=2024)
    dk = nat.DeviceKey(2048, n, p, q, h, device=0, win_bits=args.win)
    L = nat.lib()
    N = args.n
    x = np.random.default_rng(0).standard_normal(N)
    seed = bytes(range(32))
    vp = lambda a: ctypes.c_void_p(a.ctypes.data)
    ex = np.empty(N, dtype=np.int32)
    st = np.empty(N, dtype=np.int32)

    def host_enc(ct):
        nat.check(L.xhe_encrypt_f64_host(dk.handle, vp(x), N, 7, 0, 0, 1, seed, 9, vp(ct), vp(ex), vp(st)), "enc")
        return ct

    def timed(fn):
        fn()
        t0 = time.time()
        for _ in range(args.reps):
            fn()
        return (time.time() - t0) / args.reps

    out = {"n": N, "win": args.win, "host_chunk": os.environ.get("XHE_HOST_CHUNK", "default")}
    out["fresh_np_empty_per_s"] = N / timed(lambda: host_enc(np.empty((N, dk.n2w), np.uint32)))
    out["fresh_nat_empty_per_s"] = N / timed(lambda: host_enc(nat.empty((N, dk.n2w), np.uint32)))
    keep = np.empty((N, dk.n2w), np.uint32)
    out["reused_buffer_per_s"] = N / timed(lambda: host_enc(keep))
    # device-resident reference: same seed/nonce -> same draws -> same words
    xd = torch.from_numpy(x).cuda()
    m = torch.empty((N, dk.nw), dtype=torch.int32, device="cuda")
    e = torch.empty(N, dtype=torch.int32, device="cuda")
    s_ = torch.empty(N, dtype=torch.int32, device="cuda")
    r = torch.empty((N, dk.rand_words), dtype=torch.int32, device="cuda")
    c = torch.empty((N, dk.n2w), dtype=torch.int32, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    nat.check(L.xhe_encode_f64(dk.handle, xd.data_ptr(), N, 7, 0, 0, m.data_ptr(), e.data_ptr(), s_.data_ptr(),
                               stream), "encode")
    nat.check(L.xhe_rand(dk.handle, seed, 9, N, r.data_ptr(), None, stream), "rand")
    nat.check(L.xhe_encrypt(dk.handle, m.data_ptr(), r.data_ptr(), N, c.data_ptr(), stream), "encrypt")
    torch.cuda.synchronize()

    def device_step():
        nat.check(L.xhe_encode_f64(dk.handle, xd.data_ptr(), N, 7, 0, 0, m.data_ptr(), e.data_ptr(), s_.data_ptr(),
                                   stream), "encode")
        nat.check(L.xhe_rand(dk.handle, seed, 9, N, r.data_ptr(), None, stream), "rand")
        nat.check(L.xhe_encrypt(dk.handle, m.data_ptr(), r.data_ptr(), N, c.data_ptr(), stream), "encrypt")
        torch.cuda.synchronize()
    out["device_resident_per_s"] = N / timed(device_step)
    out["host_equals_device"] = bool(np.array_equal(c.cpu().numpy().view(np.uint32), keep)
                                     and np.array_equal(e.cpu().numpy(), ex))
    ctx = PaillierContext().init(p, q, djn_h_pow_n=h)
    ctx._dev = {0: dk}
    x32 = x.astype(np.float32)
    hold = {}

    def api_enc():
        hold.pop(0, None)
        hold[0] = Paillier.encrypt(ctx, x32, precision=7)
    out["dropin_encrypt_per_s"] = N / timed(api_enc)

    def api_enc_ser():
        hold.pop(1, None)
        hold[1] = Paillier.serialize(Paillier.encrypt(ctx, x32, precision=7), compression=False)
    out["dropin_encrypt_serialize_per_s"] = N / timed(api_enc_ser)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
