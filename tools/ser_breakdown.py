"""Where the label trainer's Paillier.serialize(Paillier.encrypt(x)) time goes
(logistic_regression/label_trainer.py:193-198, paillier.py:244-258): encrypt,
the D2H download, the native pickle encode (into a fresh bytes object and
into a reused, already-faulted buffer), the zstd raw frame, and the whole
chain, each timed alone on 1 M float32 (precision 7). Every rep releases the
previous rep's result first, as a training loop does.
    python tools/ser_breakdown.py [--n 1048576]"""
import argparse
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import numpy as np
    import torch
    torch.cuda.init()
    import bench
    from xfl_amd import _native as nat
    from xfl_amd import compat
    from xfl_amd.paillier import Paillier, PaillierContext
    from xfl_amd.paillier import wire
    p, q, n, h = bench.make_key(2048, seed=2024)
    ctx = PaillierContext().init(p, q, djn_h_pow_n=h)
    x = np.random.default_rng(0).standard_normal(args.n).astype(np.float32)
    rec = {"n": args.n}
    keep = {}

    def t(name, fn):
        keep.pop(name, None)
        keep[name] = fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(args.reps):
            keep.pop(name, None)
            t0 = time.time()
            keep[name] = fn()
            torch.cuda.synchronize()
            ts.append(time.time() - t0)
        rec[name + "_ms"] = min(ts) * 1e3
        return keep[name]
    enc = t("encrypt", lambda: Paillier.encrypt(ctx, x, precision=7))
    rec["window_bits"] = ctx._dev[torch.cuda.current_device()].win_bits

    def dl():
        enc._st.h = None
        return enc.words
    w = np.array(t("download", dl))
    e = enc.exponents
    raw = t("wire_encode_fresh_bytes", lambda: wire.encode_words(w, e, enc.shape))
    buf = np.empty(len(raw) + 64, np.uint8)
    buf[:] = 0
    L = nat.lib()
    shp = np.array(enc.shape, np.int64)
    need = ctypes.c_int64()
    vp = lambda a: ctypes.c_void_p(a.ctypes.data)  # noqa: E731
    t("wire_encode_warm_buffer", lambda: nat.check(L.xhe_wire_encode(vp(w), vp(e), w.shape[0], w.shape[1], vp(shp), 1,
                                                                      vp(buf), buf.shape[0], ctypes.byref(need))))
    t("zstd_raw_frame", lambda: compat.compress(raw))
    t("serialize_nocomp", lambda: (dl(), Paillier.serialize(enc, compression=False))[1])
    t("serialize_zstd", lambda: (dl(), Paillier.serialize(enc, compression=True))[1])
    # the zstd chain step by step, each rep releasing the previous one's buffers
    steps = []
    for _ in range(args.reps + 1):
        keep.clear()
        t0 = time.time()
        ww = dl()
        t1 = time.time()
        pk = wire.encode_words(ww, e, enc.shape)
        t2 = time.time()
        fr = compat.compress(pk)
        t3 = time.time()
        del pk
        t4 = time.time()
        del fr
        t5 = time.time()
        steps.append([(t1 - t0) * 1e3, (t2 - t1) * 1e3, (t3 - t2) * 1e3, (t4 - t3) * 1e3, (t5 - t4) * 1e3])
    rec["zstd_chain_steps_ms"] = {"download, encode, frame, free pickle, free frame": steps}
    keep.clear()
    out = t("encrypt_serialize_zstd", lambda: Paillier.serialize(Paillier.encrypt(ctx, x, precision=7)))
    rec["encrypt_serialize_zstd_per_s"] = args.n / rec["encrypt_serialize_zstd_ms"] * 1e3
    back = Paillier.decrypt(ctx, Paillier.ciphertext_from(ctx, out))
    rec["roundtrip_ok"] = bool(np.allclose(back, x, atol=1e-6))
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
