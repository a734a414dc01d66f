"""BASELINE.json configs 2-5 on one MI355X (the per-GPU shard of the 8-GPU
configs 4 and 5), device-resident, each checked where a cheap exact property
exists. One JSON line per config; bench.py stays the headline (config 2's
encryption at 1 M elements).

  cfg2  2048-bit, 1 M float64: encrypt -> decrypt round trip (precision None
        and 7), m recovered bit-exactly (the decode is covered by the parity
        tests against the reference's fixtures)
  cfg3  2048-bit, 10 M float32 gradient x 1e-2, precision 7: encrypt, pairwise
        homomorphic sum c_i * d_i with a second encrypted vector, and the full
        reduction prod c_i; checked by decrypting samples of the pairwise sums
  cfg4  3072-bit, 4 M elements / 8 GPUs = 500 k per GPU: encrypt (the 8-GPU job
        adds the RCCL all-gather, bench.py --key-bits 3072)
  cfg5  SecureBoost histogram: 100 k samples (12.5 k per GPU at 8 GPUs, here
        all 100 k on one), grad/hess packed by paillier_acceleration.embed,
        encrypted with precision 0, 64 features x 256 bins as ONE segmented
        product, then decrypt + umbed of the 16,384 bins; checked exactly
        against integer bin sums of the packed values

    python tools/bench_configs.py [--only cfg2,cfg5] [--steps 3] [--gpus N]

--gpus N runs cfg5 as N ranks (shard the samples, merge the partial bins);
config 4's 8-GPU form is bench.py --key-bits 3072 --n 500000 --gpus 8.
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def _sync():
    import torch
    torch.cuda.synchronize()


def _timed(fn, reps):
    fn()
    _sync()
    t = time.time()
    for _ in range(reps):
        fn()
    _sync()
    return (time.time() - t) / reps


def _key(bits, win):
    from bench import make_key
    from xfl_amd import _native as nat
    p, q, n, h = make_key(bits, seed=2024)
    t = time.time()
    dk = nat.DeviceKey(bits, n, p, q, h, device=0, win_bits=win)
    _sync()
    return dk, (p, q, n, h), time.time() - t


def _encrypt_f64(nat, L, dk, x, prec, m, ex, st, rnd, ct, nonce, stream):
    n = x.shape[0]
    nat.check(L.xhe_encode_f64(dk.handle, x.data_ptr(), n, prec, 0, 0, m.data_ptr(), ex.data_ptr(), st.data_ptr(),
                               stream), "encode")
    nat.check(L.xhe_rand(dk.handle, b"\x07" * 32, nonce, n, rnd.data_ptr(), None, stream), "rand")
    nat.check(L.xhe_encrypt(dk.handle, m.data_ptr(), rnd.data_ptr(), n, ct.data_ptr(), stream), "encrypt")


def cfg2(steps):
    import torch
    from xfl_amd import _native as nat
    L = nat.lib()
    dk, _, tk = _key(2048, 22)
    N = 1_000_000
    x = torch.from_numpy(np.random.default_rng(0).standard_normal(N)).cuda()
    m = torch.empty((N, dk.nw), dtype=torch.int32, device="cuda")
    m2 = torch.empty_like(m)
    ex = torch.empty(N, dtype=torch.int32, device="cuda")
    st = torch.empty_like(ex)
    rnd = torch.empty((N, dk.rand_words), dtype=torch.int32, device="cuda")
    ct = torch.empty((N, dk.n2w), dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    out = {"config": "cfg2: 2048-bit, 1M float64, encrypt->decrypt round trip", "key_setup_s": tk}
    for prec in (-1, 7):
        def rt():
            _encrypt_f64(nat, L, dk, x, prec, m, ex, st, rnd, ct, 1, s)
            nat.check(L.xhe_decrypt(dk.handle, ct.data_ptr(), N, m2.data_ptr(), s), "decrypt")
        t = _timed(rt, steps)
        tag = "precision_none" if prec < 0 else "precision_7"
        out[tag] = {"roundtrips_per_s": N / t, "m_bit_exact": bool(torch.equal(m, m2)),
                    "encode_status_ok": bool((st == 0).all().item())}
    return out


def cfg3(steps):
    import torch
    from xfl_amd import _native as nat
    L = nat.lib()
    dk, (p, q, n, h), tk = _key(2048, 22)
    N = 10_000_000
    g = (np.random.default_rng(1).standard_normal(N).astype(np.float32) * np.float32(1e-2)).astype(np.float64)
    x = torch.from_numpy(g).cuda()
    m = torch.empty((N, dk.nw), dtype=torch.int32, device="cuda")
    ex = torch.empty(N, dtype=torch.int32, device="cuda")
    st = torch.empty_like(ex)
    rnd = torch.empty((N, dk.rand_words), dtype=torch.int32, device="cuda")
    c = torch.empty((N, dk.n2w), dtype=torch.int32, device="cuda")
    d = torch.empty_like(c)
    cd = torch.empty_like(c)
    s = torch.cuda.current_stream().cuda_stream
    _encrypt_f64(nat, L, dk, x, 7, m, ex, st, rnd, d, 99, s)  # the second encrypted vector
    md = m.clone()
    t_enc = _timed(lambda: _encrypt_f64(nat, L, dk, x, 7, m, ex, st, rnd, c, 1, s), steps)
    t_add = _timed(lambda: nat.check(L.xhe_mulmod(dk.handle, c.data_ptr(), None, d.data_ptr(), None, N, 0,
                                                  cd.data_ptr(), None, s), "add"), steps)
    seg = np.array([0, N], dtype=np.int64)
    tot = torch.empty((1, dk.n2w), dtype=torch.int32, device="cuda")
    t_red = _timed(lambda: nat.check(L.xhe_segprod(dk.handle, c.data_ptr(), None, 0, N, seg.ctypes.data_as(
        ctypes.c_void_p), 1, tot.data_ptr(), s), "reduce"), max(1, steps // 2))
    # check: decrypt a sample of pairwise sums; plaintexts add mod n
    idx = torch.tensor([0, 1, N // 3, N - 1], device="cuda")
    mm = torch.empty((4, dk.nw), dtype=torch.int32, device="cuda")
    nat.check(L.xhe_decrypt(dk.handle, cd[idx].contiguous().data_ptr(), 4, mm.data_ptr(), s), "decrypt")
    _sync()
    w = lambda a: nat.words_to_ints(a.cpu().numpy().view(np.uint32))  # noqa: E731
    ok = all(v == (a + b) % n for v, a, b in zip(w(mm), w(m[idx]), w(md[idx])))
    return {"config": "cfg3: 2048-bit, 10M float32 gradient, encrypt + pairwise sum + reduction",
            "encrypts_per_s": N / t_enc, "pairwise_adds_per_s": N / t_add, "reduction_10M_s": t_red,
            "pairwise_sample_bit_exact": ok, "key_setup_s": tk}


def cfg4(steps):
    import torch
    from xfl_amd import _native as nat
    L = nat.lib()
    # the window policy of bench.py and the key-size table (bench.pick_window:
    # the uniform window with the fewest table products leaving 16 GiB free)
    from bench import pick_window
    win = pick_window(3072, torch.cuda.mem_get_info(0)[0])
    dk, _, tk = _key(3072, win)
    N = 500_000
    x = torch.from_numpy(np.random.default_rng(2).standard_normal(N)).cuda()
    m = torch.empty((N, dk.nw), dtype=torch.int32, device="cuda")
    m2 = torch.empty_like(m)
    ex = torch.empty(N, dtype=torch.int32, device="cuda")
    st = torch.empty_like(ex)
    rnd = torch.empty((N, dk.rand_words), dtype=torch.int32, device="cuda")
    ct = torch.empty((N, dk.n2w), dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    t = _timed(lambda: _encrypt_f64(nat, L, dk, x, 7, m, ex, st, rnd, ct, 1, s), steps)
    nat.check(L.xhe_decrypt(dk.handle, ct.data_ptr(), N, m2.data_ptr(), s), "decrypt")
    _sync()
    return {"config": "cfg4: 3072-bit, 500k elements (one GPU's shard of 4M over 8)", "encrypts_per_s": N / t,
            "roundtrip_bit_exact": bool(torch.equal(m, m2)), "fixed_base_window_bits": win, "key_setup_s": tk}


def cfg5(steps, world=1, rank=0):
    """Config 5. With world > 1 each rank takes a contiguous shard of the
    samples (12.5 k of 100 k at 8 ranks), encrypts it, builds its 64 x 256 local
    bins with one segmented product, and the ranks' partial bins are merged by
    shard.merge_segment_products (all-gather of the partials + one device
    combine per bin: xgb_actor.py:447-455 merge_hist, decision_tree_trainer.py:
    170-183). Rank 0 decrypts the merged bins and checks them exactly."""
    import torch
    import torch.distributed as dist
    from xfl_amd import _native as nat
    from xfl_amd.paillier_acceleration import embed, umbed
    from xfl_amd.shard import device_combine, merge_segment_products, shard_range
    L = nat.lib()
    dk, (p, q, n, h), tk = _key(2048, 22)
    S, F, NB = 100_000, 64, 256
    rng = np.random.default_rng(3)
    z = rng.standard_normal(S)
    y = (rng.random(S) < 0.5).astype(np.float64)
    pr = 1.0 / (1.0 + np.exp(-z))
    gr, he = pr - y, pr * (1.0 - pr)
    bins = np.stack([np.random.default_rng(4 + f).integers(0, NB, S) for f in range(F)])
    lo, hi, _ = shard_range(S, world, rank)
    Sl = hi - lo
    t = time.time()
    packed = embed([gr[lo:hi], he[lo:hi]])  # reference semantics (paillier_acceleration.py:21-32)
    t_embed = time.time() - t
    mw = nat.ints_to_words([int(v) % n for v in packed], dk.nw)
    mdev = torch.from_numpy(mw.view(np.int32)).cuda()
    rnd = torch.empty((Sl, dk.rand_words), dtype=torch.int32, device="cuda")
    ct = torch.empty((Sl, dk.n2w), dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream

    def enc():
        nat.check(L.xhe_rand(dk.handle, b"\x05" * 32, 3 + rank, Sl, rnd.data_ptr(), None, s), "rand")
        nat.check(L.xhe_encrypt(dk.handle, mdev.data_ptr(), rnd.data_ptr(), Sl, ct.data_ptr(), s), "encrypt")
    t_enc = _timed(enc, steps)
    lbins = bins[:, lo:hi]
    bins_d = torch.from_numpy(np.ascontiguousarray(lbins)).cuda()
    order = torch.argsort(bins_d, dim=1, stable=True)  # per feature, samples grouped by bin
    counts = np.stack([np.bincount(lbins[f], minlength=NB) for f in range(F)]).reshape(-1)
    seg = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
    local = torch.empty((F * NB, dk.n2w), dtype=torch.int32, device="cuda")
    zeros = torch.zeros(F * NB, dtype=torch.int32, device="cuda")  # precision 0: every exponent is 0
    counts_d = torch.from_numpy(counts).cuda()
    combine = device_combine(dk)
    merged = {}

    def build():
        gathered = ct.index_select(0, order.reshape(-1))  # [F*Sl, n2w], feature-major, bin-ordered
        nat.check(L.xhe_segprod(dk.handle, gathered.data_ptr(), None, 0, F * Sl, seg.ctypes.data_as(
            ctypes.c_void_p), F * NB, local.data_ptr(), s), "hist")
        if world > 1:
            merged["h"], _, merged["c"] = merge_segment_products(local, zeros, combine, counts=counts_d)
        else:
            merged["h"], merged["c"] = local, counts_d

    if world > 1:
        dist.barrier()
    t_hist = _timed(build, steps)
    if world > 1:
        t_hist = max_over_ranks(t_hist)
        t_enc = max_over_ranks(t_enc)
    hist = merged["h"]
    rec = {"config": "cfg5: SecureBoost histogram 100k samples x 64 features x 256 bins (packed grad/hess)",
           "ranks": world, "samples_per_rank": Sl, "embed_s": t_embed, "encrypt_per_s": S / t_enc if world > 1
           else Sl / t_enc, "histogram_64x256_s": t_hist, "sample_features_per_s": S * F / t_hist, "key_setup_s": tk}
    if rank != 0:
        return None
    # decrypt + umbed every bin (label side, decision_tree_label_trainer.py:245-293)
    mh = torch.empty((F * NB, dk.nw), dtype=torch.int32, device="cuda")
    t = time.time()
    nat.check(L.xhe_decrypt(dk.handle, hist.data_ptr(), F * NB, mh.data_ptr(), s), "decrypt")
    _sync()
    vals = [v - n if v >= n - n // 3 else v for v in nat.words_to_ints(mh.cpu().numpy().view(np.uint32))]
    g_sum, h_sum = umbed(vals, 2)
    t_dec = time.time() - t
    # exact check on 4 features: integer bin sums of int(g 2^64), int(h 2^64) over ALL samples
    gi = [int(v * (1 << 64)) for v in gr]
    hi_ = [int(v * (1 << 64)) for v in he]
    ok = bool(np.array_equal(merged["c"].cpu().numpy(),
                             np.stack([np.bincount(bins[f], minlength=NB) for f in range(F)]).reshape(-1)))
    for f in (0, 17, 40, 63):
        gs, hs = [0] * NB, [0] * NB
        for i, b in enumerate(bins[f]):
            gs[b] += gi[i]
            hs[b] += hi_[i]
        ok &= all(np.float32(gs[b] / (1 << 64)) == g_sum[f * NB + b] and np.float32(hs[b] / (1 << 64)) == h_sum[f * NB + b]
                  for b in range(NB))
    rec.update({"decrypt_umbed_16384_bins_s": t_dec, "bins_bit_exact_4_features": bool(ok)})
    return rec


def max_over_ranks(v):
    import torch
    import torch.distributed as dist
    t = torch.tensor([v], dtype=torch.float64)
    if dist.get_backend() == "nccl":
        t = t.cuda()
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="cfg2,cfg3,cfg4,cfg5")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks for cfg5 (one process per GPU; ranks beyond the visible GPUs share them over gloo)")
    args = ap.parse_args()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        from xfl_amd.shard import spawn_local_ranks
        sys.exit(spawn_local_ranks(args.gpus, [os.path.abspath(__file__)] + sys.argv[1:]))
    import torch
    world = int(env_world or "1")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = torch.cuda.device_count()
    torch.cuda.set_device(local % ndev)
    if world > 1:
        import torch.distributed as dist
        if world <= ndev:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:  # rehearsal with more ranks than GPUs: RCCL needs one GPU per rank
            dist.init_process_group("gloo")
    fns = {"cfg2": cfg2, "cfg3": cfg3, "cfg4": cfg4, "cfg5": cfg5}
    for name in args.only.split(","):
        if world > 1 and name != "cfg5":
            continue  # cfg4's multi-GPU form is bench.py --key-bits 3072 --n 500000 --gpus 8
        rec = fns[name](args.steps, world, rank) if name == "cfg5" else fns[name](args.steps)
        if rec is not None:
            print(json.dumps(rec), flush=True)
        torch.cuda.empty_cache()
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
