"""Multi-rank paths on CPU with gloo (world size 2-3): the bench's
step -> async all-gather -> drain -> parity flow (xfl_amd.shard.GatherPipeline
+ shard_parity, exactly what bench.py --gpus N runs) on oracle-encrypted
shards, and the partial-histogram merge (merge_segment_products, the analogue
of xgb_actor.merge_hist, core/tree_ray/xgb_actor.py:447-456) on the reference's
golden histogram."""
import os
import random
import subprocess
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tests.conftest import FIXTURES, ROOT, hx, load_fixture


def _run(target, world, *args):
    from xfl_amd.shard import free_port
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q) + args) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    return dict(res)


def _init(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    sys.path.insert(0, ROOT)
    dist.init_process_group("gloo", rank=rank, world_size=world)


def _gather_worker(rank, world, port, q, n, words):
    _init(rank, world, port)
    from xfl_amd.shard import gather_rows, pad_rows, shard_range
    lo, hi, per = shard_range(n, world, rank)
    full = torch.arange(n * words, dtype=torch.int32).reshape(n, words)
    local = pad_rows(full[lo:hi], per)
    out = gather_rows(local, world * per)
    rows = torch.cat([out[r * per: r * per + (shard_range(n, world, r)[1] - shard_range(n, world, r)[0])]
                      for r in range(world)], 0)
    q.put((rank, bool(torch.equal(rows, full))))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n", [(2, 7), (2, 8), (3, 10)])
def test_gather_reassembles_vector(world, n):
    res = _run(_gather_worker, world, n, 4)
    assert all(res.values())


def test_shard_range_covers():
    from xfl_amd.shard import shard_range
    for n in (0, 1, 7, 1000):
        for w in (1, 2, 3, 8):
            seen = []
            for r in range(w):
                lo, hi, _ = shard_range(n, w, r)
                seen.extend(range(lo, hi))
            assert seen == list(range(n))


# ------------------------------------------------------------ bench flow
ROWS = 3


def _shard_inputs(okey, rank, step):
    """The rank's plaintexts (seeded by rank, like bench.py) and the step's
    obfuscation draws (seeded by step and global element position)."""
    xs = np.random.default_rng(rank).standard_normal(ROWS)
    rs = [random.Random(step * 1000 + rank * ROWS + i).randrange(1, okey["djn_exp_bound"]) for i in range(ROWS)]
    return xs, rs


def _expected_shard(O, okey, rank, step):
    xs, rs = _shard_inputs(okey, rank, step)
    return [O.encrypt_m(okey, O.encode_element(okey, float(x), 7)[0], r) for x, r in zip(xs, rs)]


def _pipeline_worker(rank, world, port, q, proxy=None):
    _init(rank, world, port)
    from oracle import paillier_oracle as O
    from xfl_amd._native import ints_to_words
    from xfl_amd.shard import GatherPipeline, shard_parity
    g = load_fixture(FIXTURES[0])
    k = g["key"]
    okey = O.derive_private(hx(k["p"]), hx(k["q"]), hx(k["h_pow_n"]))
    n2w = g["key_bits"] // 16

    def produce(i, buf):  # the bench's encode + draw + encrypt, as the oracle computes it
        buf.copy_(torch.from_numpy(ints_to_words(_expected_shard(O, okey, rank, i), n2w).view(np.int32).copy()))

    pipe = GatherPipeline(produce, ROWS, n2w, world=world, rank=rank, device="cpu", proxy_world=proxy)
    for i in range(5):  # warmup 2 + timed 3 with the double buffer wrapping around
        pipe.step(i)
    pipe.drain()
    last = 4
    want = torch.cat([torch.from_numpy(ints_to_words(_expected_shard(O, okey, r, last), n2w).view(np.int32).copy())
                      for r in range(world)])
    ok_vec = bool(torch.equal(pipe.vector(last), want))
    expected = lambda i: _expected_shard(O, okey, rank, last)[i]  # noqa: E731
    ok_parity = shard_parity(pipe.shard(last), pipe.vector(last), rank, [0, ROWS - 1], expected)
    # the parity check must fail on a wrong shard or a wrong reassembly
    bad = lambda i: _expected_shard(O, okey, rank, last - 1)[i]  # noqa: E731
    ok_neg = not shard_parity(pipe.shard(last), pipe.vector(last), rank, [0], bad)
    other = pipe.vector(last).clone()
    other[rank * ROWS] += 1
    ok_neg = ok_neg and not shard_parity(pipe.shard(last), other, rank, [1], expected)
    if proxy:  # the gather targets are sized for `proxy` ranks
        ok_vec = ok_vec and all(g.shape[0] == proxy * ROWS for g in pipe.gathered)
    q.put((rank, (ok_vec, ok_parity, ok_neg)))
    dist.destroy_process_group()


@pytest.mark.parametrize("proxy", [None, 8])
def test_bench_pipeline_world2(proxy):
    """proxy=8: bench.py --proxy-world, the 8-rank gather volume and target
    size issued from 2 ranks; the real vector is unaffected."""
    res = _run(_pipeline_worker, 2, proxy)
    for r, (ok_vec, ok_parity, ok_neg) in res.items():
        assert ok_vec, f"rank {r}: reassembled vector != all ranks' oracle encryptions"
        assert ok_parity and ok_neg, f"rank {r}: shard_parity"


def test_bench_refuses_mismatched_world():
    env = dict(os.environ, WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "must agree" in r.stderr


# ------------------------------------------------------------ histogram merge
def _oracle_combine(okey):
    n2 = okey["n_square"]

    def combine(words, d, seg_begin):
        from xfl_amd._native import ints_to_words, words_to_ints
        vals = words_to_ints(words.numpy().view(np.uint32))
        dd = d.tolist()
        out = []
        for s in range(len(seg_begin) - 1):
            acc = 1
            for i in range(int(seg_begin[s]), int(seg_begin[s + 1])):
                acc = acc * pow(vals[i], 1 << dd[i], n2) % n2
            out.append(acc)
        return torch.from_numpy(ints_to_words(out, words.shape[1]).view(np.int32).copy())
    return combine


def _local_partials(O, okey, raws, exps, bins, nbins):
    """This rank's groupby(bin).sum(): per-bin aligned products (empty bin:
    1 with exponent 0, the reference's fillna(0) + add)."""
    parts, pe, cnt = [], [], []
    for b in range(nbins):
        idx = [i for i in range(len(raws)) if bins[i] == b]
        if idx:
            r, e = O.sum_ct(okey, [raws[i] for i in idx], [exps[i] for i in idx])
        else:
            r, e = 1, 0
        parts.append(r)
        pe.append(e)
        cnt.append(len(idx))
    return parts, pe, cnt


def _merge_worker(rank, world, port, q, case):
    _init(rank, world, port)
    from oracle import paillier_oracle as O
    from xfl_amd._native import ints_to_words, words_to_ints
    from xfl_amd.shard import merge_segment_products, shard_range
    g = load_fixture(FIXTURES[0])
    k = g["key"]
    okey = O.derive_private(hx(k["p"]), hx(k["q"]), hx(k["h_pow_n"]))
    n2w = g["key_bits"] // 16
    if case == "hist":
        h = g["ops"]["hist"]
        raws, exps, bins, nb = [hx(r) for r in h["ct"]["raw"]], h["ct"]["exp"], h["bins"], len(h["bin_ids"])
        want = ([hx(r) for r in h["sum"]["raw"]], h["sum"]["exp"], h["count"])
    else:  # mixed exponents: np.sum over ops.a split across ranks
        a = g["ops"]["a"]
        raws, exps, nb = [hx(r) for r in a["raw"]], a["exp"], 1
        bins = [0] * len(raws)
        want = ([hx(r) for r in g["ops"]["sum_a"]["raw"]], g["ops"]["sum_a"]["exp"], [len(raws)])
    lo, hi, _ = shard_range(len(raws), world, rank)
    parts, pe, cnt = _local_partials(O, okey, raws[lo:hi], exps[lo:hi], bins[lo:hi], nb)
    out, eout, counts = merge_segment_products(
        torch.from_numpy(ints_to_words(parts, n2w).view(np.int32).copy()), torch.tensor(pe, dtype=torch.int32),
        _oracle_combine(okey), counts=torch.tensor(cnt, dtype=torch.int64))
    got = (words_to_ints(out.numpy().view(np.uint32)), eout.tolist(), counts.tolist())
    q.put((rank, got == want))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("case", ["hist", "mixed_exp_sum"])
def test_merge_segment_products(world, case):
    """Per-rank partial bins, all-gathered and combined per bin, equal the
    reference's single-process groupby sum / np.sum bit for bit."""
    res = _run(_merge_worker, world, case)
    assert all(res.values()), res
