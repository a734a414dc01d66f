"""Multi-rank sharding + reassembly (the N>1 bench path) on CPU with gloo."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, words, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from xfl_amd.shard import gather_rows, pad_rows, shard_range
    lo, hi, per = shard_range(n, world, rank)
    full = torch.arange(n * words, dtype=torch.int32).reshape(n, words)
    local = pad_rows(full[lo:hi], per)
    out = gather_rows(local, world * per)
    # drop the padding of each shard
    rows = torch.cat([out[r * per: r * per + (shard_range(n, world, r)[1] - shard_range(n, world, r)[0])]
                      for r in range(world)], 0)
    q.put((rank, bool(torch.equal(rows, full))))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n", [(2, 7), (2, 8), (3, 10)])
def test_gather_reassembles_vector(world, n):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, 4, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(ok for _, ok in res)


def test_shard_range_covers():
    from xfl_amd.shard import shard_range
    for n in (0, 1, 7, 1000):
        for w in (1, 2, 3, 8):
            seen = []
            for r in range(w):
                lo, hi, _ = shard_range(n, w, r)
                seen.extend(range(lo, hi))
            assert seen == list(range(n))
