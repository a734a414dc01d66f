"""Multi-rank histogram merge with the device combine (xhe_segprod), on one GPU:
world-1 in process, and two gloo ranks sharing cuda:0 (each computes its
partial bins on the device, the partials travel through gloo, the per-bin
combine runs on the device). Equal to the reference's groupby sum bit for bit
(tests/golden ops.hist; decision_tree_trainer.py:151-183, xgb_actor.py:447-456)."""
import os
import sys

import numpy as np
import pytest
import torch

from tests.conftest import FIXTURES, ROOT, hx, load_fixture

pytestmark = pytest.mark.gpu


def _case(g):
    h = g["ops"]["hist"]
    return ([hx(r) for r in h["ct"]["raw"]], h["ct"]["exp"], h["bins"], len(h["bin_ids"]),
            ([hx(r) for r in h["sum"]["raw"]], h["sum"]["exp"], h["count"]))


def _dkey(g):
    from xfl_amd._native import DeviceKey
    k = g["key"]
    return DeviceKey(g["key_bits"], hx(k["n"]), None, None, None)


def _local_partials_device(dk, raws, exps, bins, nb):
    """groupby(bin).sum() of this rank's samples on the device: samples
    ordered by bin, one xhe_segprod (empty bins give 1, exponent 0)."""
    from xfl_amd import _native as nat
    from xfl_amd.shard import device_combine
    order = sorted(range(len(raws)), key=lambda i: bins[i])
    counts = np.bincount(np.asarray(bins, dtype=np.int64), minlength=nb) if bins else np.zeros(nb, np.int64)
    seg = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
    e = np.asarray([exps[i] for i in order], dtype=np.int64)
    emin = np.array([e[seg[s]:seg[s + 1]].min() if seg[s + 1] > seg[s] else 0 for s in range(nb)], dtype=np.int64)
    d = np.concatenate([e[seg[s]:seg[s + 1]] - emin[s] for s in range(nb)]).astype(np.int32) if len(e) else \
        np.zeros(0, np.int32)
    words = torch.from_numpy(nat.ints_to_words([raws[i] for i in order] or [1], dk.n2w).view(np.int32).copy()).cuda()
    out = device_combine(dk)(words[:len(order)] if order else words[:0], torch.from_numpy(d).cuda(), seg)
    return out, torch.from_numpy(emin.astype(np.int32)).cuda(), torch.from_numpy(counts).cuda()


def test_merge_world1_device():
    from xfl_amd import _native as nat
    from xfl_amd.shard import device_combine, merge_segment_products
    g = load_fixture(FIXTURES[0])
    dk = _dkey(g)
    raws, exps, bins, nb, want = _case(g)
    parts, pe, cnt = _local_partials_device(dk, raws, exps, bins, nb)
    out, eout, counts = merge_segment_products(parts, pe, device_combine(dk), counts=cnt)
    torch.cuda.synchronize()
    assert (nat.words_to_ints(out.cpu().numpy().view(np.uint32)), eout.tolist(), counts.tolist()) == want


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    sys.path.insert(0, ROOT)
    import torch.distributed as dist

    from xfl_amd import _native as nat
    from xfl_amd.shard import device_combine, merge_segment_products, shard_range
    torch.cuda.init()
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = load_fixture(FIXTURES[0])
    dk = _dkey(g)
    raws, exps, bins, nb, want = _case(g)
    lo, hi, _ = shard_range(len(raws), world, rank)
    parts, pe, cnt = _local_partials_device(dk, raws[lo:hi], exps[lo:hi], bins[lo:hi], nb)
    out, eout, counts = merge_segment_products(parts, pe, device_combine(dk), counts=cnt)
    torch.cuda.synchronize()
    got = (nat.words_to_ints(out.cpu().numpy().view(np.uint32)), eout.tolist(), counts.tolist())
    q.put((rank, got == want))
    dist.destroy_process_group()


def test_merge_two_gloo_ranks_device_combine():
    import torch.multiprocessing as mp

    from xfl_amd.shard import free_port
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert all(res.values()), res


# ------------------------------------------------------------ drop-in sharding
def test_dropin_shards_over_devices(monkeypatch):
    """num_cores / $XHE_DEVICES spread a batch over GPUs (the reference's
    process pool, paillier.py:321-332,388-394): three shards on device 0 here,
    each a host thread with its own slice of the output. Deterministic ops
    equal the single-shard result bit for bit; encryptions decrypt back and
    each shard draws its own randomness."""
    from tests import dropin_cases as C
    from xfl_amd.paillier import Paillier, ops
    priv, pub = C.ctxs(load_fixture(FIXTURES[0]))
    rng = np.random.default_rng(4)
    x = (rng.random(3001) * 100 - 50).astype(np.float32)
    y = rng.standard_normal(3001)
    monkeypatch.setenv("XHE_DEVICES", "0")
    c1 = Paillier.encrypt(priv, x, precision=7)
    want_add = c1 + c1
    want_mul = c1 * y
    want_dec = Paillier.decrypt(priv, c1)
    monkeypatch.setenv("XHE_DEVICES", "0,0,0")
    monkeypatch.setattr(ops, "MIN_SHARD", 512)
    calls = []
    real = ops.sharded

    def spy(ctx, count, body, num_cores=-1):
        calls.append((count, len(ctx.shard_devices(num_cores))))
        return real(ctx, count, body, num_cores)
    monkeypatch.setattr(ops, "sharded", spy)
    assert C.raw(c1 + c1) == C.raw(want_add)
    assert C.raw(c1 * y) == C.raw(want_mul)
    assert np.array_equal(Paillier.decrypt(priv, c1), want_dec)
    c3 = Paillier.encrypt(pub, x, precision=7)
    assert np.all(np.abs(Paillier.decrypt(priv, c3) - x) < 1e-4)
    w = c3.words
    third = len(x) // 3
    assert len({w[i].tobytes() for i in (0, third, 2 * third)}) == 3
    # same plaintext in every shard: distinct draws per shard
    same = Paillier.encrypt(priv, np.full(3000, 1.25), precision=7)
    assert len({bytes(r) for r in same.words}) == 3000
    assert calls and all(d == 3 for _, d in calls)
