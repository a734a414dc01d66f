"""Config 4's reassembly path on the GPU (BASELINE.json configs[3]: 3072-bit
key, elements sharded over ranks, ciphertext shards all-gathered into the
whole vector). The shard producer is the bench's own step - device encode
(xhe_encode_f64) + ChaCha20 draws (xhe_rand) + DJN-CRT encryption
(xhe_encrypt), bench.py encrypt_shard - driven by shard.GatherPipeline on the
3072-bit fixture key:

* world 1 in process, the pipeline's vector on cuda:0;
* two gloo ranks sharing cuda:0: each encrypts its shard on the device and the
  pipeline gathers through host memory (gloo moves CPU tensors; on an 8-GPU
  node the same pipeline runs RCCL over device tensors, bench.py).

The reassembled vector must equal the oracle's encryptions of every rank's
plaintexts with the draws the device made (the reference encrypts the same
elements in a process pool, paillier.py:321-332), and shard_parity must reject
a perturbed shard and a perturbed reassembly."""
import os
import sys

import numpy as np
import pytest
import torch

from tests.conftest import ROOT, hx, load_fixture

pytestmark = pytest.mark.gpu

FIX = "paillier_3072_djn.json"
ROWS = 1000          # elements per rank per step
SAMPLE = (0, 1, 499, 998, 999)


def _key():
    from xfl_amd._native import DeviceKey
    g = load_fixture(FIX)
    k = g["key"]
    p, q, h = hx(k["p"]), hx(k["q"]), hx(k["h_pow_n"])
    return DeviceKey(g["key_bits"], p * q, p, q, h, device=0, win_bits=12), (p, q, h)


class _Encryptor:
    """bench.py encrypt_shard for one rank: x resident on the device, a fresh
    seed per rank, nonce = step."""

    def __init__(self, dk, rank):
        from xfl_amd import _native as nat
        self.nat, self.L, self.dk = nat, nat.lib(), dk
        self.xs = np.random.default_rng(100 + rank).standard_normal(ROWS) * 1e3
        self.x = torch.from_numpy(self.xs).cuda()
        self.m = torch.empty((ROWS, dk.nw), dtype=torch.int32, device="cuda")
        self.ex = torch.empty(ROWS, dtype=torch.int32, device="cuda")
        self.st = torch.empty(ROWS, dtype=torch.int32, device="cuda")
        self.rnd = torch.empty((ROWS, dk.rand_words), dtype=torch.int32, device="cuda")
        self.seed = bytes([rank + 1]) * 32

    def draws(self, step):
        """the step's draws (a fresh xhe_rand of the same stream)"""
        r = torch.empty_like(self.rnd)
        s = torch.cuda.current_stream().cuda_stream
        self.nat.check(self.L.xhe_rand(self.dk.handle, self.seed, step, ROWS, r.data_ptr(), None, s), "rand")
        torch.cuda.synchronize()
        return r.cpu().numpy().view(np.uint32)

    def __call__(self, i, ct):
        nat, L, dk = self.nat, self.L, self.dk
        s = torch.cuda.current_stream().cuda_stream
        nat.check(L.xhe_encode_f64(dk.handle, self.x.data_ptr(), ROWS, 7, 0, 0, self.m.data_ptr(),
                                   self.ex.data_ptr(), self.st.data_ptr(), s), "encode")
        nat.check(L.xhe_rand(dk.handle, self.seed, i, ROWS, self.rnd.data_ptr(), None, s), "rand")
        nat.check(L.xhe_encrypt(dk.handle, self.m.data_ptr(), self.rnd.data_ptr(), ROWS, ct.data_ptr(), s),
                  "encrypt")


def _expected(okey, enc, step, i, draws=None):
    from oracle import paillier_oracle as O
    from xfl_amd._native import words_to_ints
    d = enc.draws(step) if draws is None else draws
    return O.encrypt_m(okey, O.encode_element(okey, float(enc.xs[i]), 7)[0], words_to_ints(d[i]))


def _ints(t):
    from xfl_amd._native import words_to_ints
    return words_to_ints(t.cpu().numpy().view(np.uint32))


def test_gather_pipeline_world1_device():
    from oracle import paillier_oracle as O
    from xfl_amd.shard import GatherPipeline, shard_parity
    dk, (p, q, h) = _key()
    okey = O.derive_private(p, q, h)
    enc = _Encryptor(dk, 0)
    pipe = GatherPipeline(enc, ROWS, dk.n2w, world=1, rank=0, device="cuda")
    for i in range(3):
        pipe.step(i)
    pipe.drain()
    torch.cuda.synchronize()
    last = 2
    vec = pipe.vector(last)
    assert vec.device.type == "cuda" and tuple(vec.shape) == (ROWS, dk.n2w)
    draws = enc.draws(last)
    got = _ints(vec[list(SAMPLE)])
    assert got == [_expected(okey, enc, last, i, draws) for i in SAMPLE]
    expected = lambda i: _expected(okey, enc, last, i, draws)  # noqa: E731
    assert shard_parity(pipe.shard(last), None, 0, [0, ROWS - 1], expected)
    bad = pipe.shard(last).clone()
    bad[ROWS - 1, 3] ^= 1
    assert not shard_parity(bad, None, 0, [ROWS - 1], expected)
    # an earlier step's draws are not this step's ciphertexts
    assert not shard_parity(pipe.shard(last), None, 0, [0], lambda i: _expected(okey, enc, 1, i))


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    sys.path.insert(0, ROOT)
    import torch.distributed as dist

    from oracle import paillier_oracle as O
    from xfl_amd.shard import GatherPipeline, shard_parity
    try:
        torch.cuda.init()
        dist.init_process_group("gloo", rank=rank, world_size=world)
        dk, (p, q_, h) = _key()
        okey = O.derive_private(p, q_, h)
        encs = [_Encryptor(dk, r) for r in range(world)]  # every rank's inputs (deterministic)
        mine = encs[rank]
        dev = torch.empty((ROWS, dk.n2w), dtype=torch.int32, device="cuda")

        def produce(i, buf):  # device encrypt, then into the host shard gloo gathers
            mine(i, dev)
            buf.copy_(dev.cpu())

        pipe = GatherPipeline(produce, ROWS, dk.n2w, world=world, rank=rank, device="cpu")
        for i in range(4):  # the double buffer wraps around
            pipe.step(i)
        pipe.drain()
        last = 3
        vec = pipe.vector(last)
        ok_vec = tuple(vec.shape) == (world * ROWS, dk.n2w)
        for r in range(world):
            draws = encs[r].draws(last)
            got = _ints(vec[[r * ROWS + i for i in SAMPLE]])
            ok_vec = ok_vec and got == [_expected(okey, encs[r], last, i, draws) for i in SAMPLE]
        draws = mine.draws(last)
        expected = lambda i: _expected(okey, mine, last, i, draws)  # noqa: E731
        ok_par = shard_parity(pipe.shard(last), vec, rank, [0, ROWS - 1], expected)
        other = vec.clone()
        other[rank * ROWS + 1, 0] ^= 1
        ok_neg = not shard_parity(pipe.shard(last), other, rank, [0], expected)
        q.put((rank, (ok_vec, ok_par, ok_neg)))
        dist.destroy_process_group()
    except Exception as exc:  # report instead of hanging the parent
        q.put((rank, repr(exc)))


def test_gather_pipeline_two_gloo_ranks_share_gpu():
    import torch.multiprocessing as mp

    from xfl_amd.shard import free_port
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    for r, v in res.items():
        assert isinstance(v, tuple), f"rank {r}: {v}"
        ok_vec, ok_par, ok_neg = v
        assert ok_vec, f"rank {r}: reassembled 3072-bit vector != oracle encryptions of every rank's shard"
        assert ok_par and ok_neg, f"rank {r}: shard_parity"
