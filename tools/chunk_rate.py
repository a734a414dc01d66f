"""Device-resident DJN encryption rate of 1 M elements issued as one launch
sequence vs as k chunks (the host pipeline's granularity), on one stream and
round-robin over three streams: python tools/chunk_rate.py [--win 23]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--win", type=int, default=23)
    args = ap.parse_args()
    import numpy as np
    import torch
    from bench import make_key
    from xfl_amd import _native as nat
    p, q, n, h = make_key(2048, seed=2024)
    dk = nat.DeviceKey(2048, n, p, q, h, device=0, win_bits=args.win)
    L = nat.lib()
    N = 1 << 20
    x = torch.from_numpy(np.random.default_rng(0).standard_normal(N)).cuda()
    m = torch.empty((N, dk.nw), dtype=torch.int32, device="cuda")
    e = torch.empty(N, dtype=torch.int32, device="cuda")
    s_ = torch.empty(N, dtype=torch.int32, device="cuda")
    r = torch.empty((N, dk.rand_words), dtype=torch.int32, device="cuda")
    c = torch.empty((N, dk.n2w), dtype=torch.int32, device="cuda")
    streams = [torch.cuda.Stream() for _ in range(3)]
    seed = bytes(32)

    def run(chunk, nstreams):
        for i, off in enumerate(range(0, N, chunk)):
            k = min(chunk, N - off)
            st = streams[i % nstreams].cuda_stream
            nat.check(L.xhe_encode_f64(dk.handle, x.data_ptr() + off * 8, k, 7, 0, 0, m.data_ptr() + off * dk.nw * 4,
                                       e.data_ptr() + off * 4, s_.data_ptr() + off * 4, st))
            nat.check(L.xhe_rand(dk.handle, seed, 1 + off, k, r.data_ptr() + off * dk.rand_words * 4, None, st))
            nat.check(L.xhe_encrypt(dk.handle, m.data_ptr() + off * dk.nw * 4, r.data_ptr() + off * dk.rand_words * 4,
                                    k, c.data_ptr() + off * dk.n2w * 4, st))
        torch.cuda.synchronize()

    out = {"win": args.win, "n": N}
    for chunk in (N, 1 << 19, 1 << 18, 1 << 17):
        for ns in ((1, 3) if chunk < N else (1,)):
            run(chunk, ns)
            t0 = time.time()
            for _ in range(3):
                run(chunk, ns)
            out[f"chunk{chunk}_streams{ns}_per_s"] = 3 * N / (time.time() - t0)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
