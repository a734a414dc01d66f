"""Element sharding across the GPUs of one node.

Encrypt/decrypt/add/scalar-mul are element-independent: rank r owns the
contiguous range [r*ceil(N/G), min(N, (r+1)*ceil(N/G))) - the reference's
analogue is the process pool over data.reshape(-1) (paillier.py:321-332,
388-394). There are exactly two exchange steps:

* reassembling the ciphertext vector: one all-gather of equally padded row
  shards (RCCL over xGMI on the GPU, `gloo` on CPU for tests), pipelined
  behind the next step's kernels (GatherPipeline);
* merging per-rank partial homomorphic sums / histograms. RCCL cannot
  reduce with a modular product, so the [nseg][n2w] partials are all-gathered
  and each bin's G partials are combined locally by one segmented product
  (merge_segment_products) - the analogue of xgb_actor.merge_hist
  (core/tree_ray/xgb_actor.py:447-456: concat + groupby(index).sum) and of
  the row-batch merge in decision_tree_trainer.py:170-183 (outer merge,
  fillna(0), +).

spawn_local_ranks() starts one process per GPU (bench.py --gpus N without
torchrun); it must run before the parent touches the GPU.
"""
import os
import socket
import subprocess
import sys
import time

import numpy as np
import torch
import torch.distributed as dist


def shard_range(n, world, rank):
    per = -(-n // world) if world else n
    lo = min(n, rank * per)
    hi = min(n, lo + per)
    return lo, hi, per


def gather_rows(local, n_total, group=None):
    """All-gather equally padded row shards ([per, words] int32) into
    [n_total, words] on every rank."""
    world = dist.get_world_size(group)
    per = local.shape[0]
    out = torch.empty((world * per,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    dist.all_gather_into_tensor(out, local.contiguous(), group=group)
    return out[:n_total]


def pad_rows(x, per):
    if x.shape[0] == per:
        return x
    pad = torch.zeros((per - x.shape[0],) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    return torch.cat([x, pad], 0)


# ------------------------------------------------------------ launching
def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def spawn_local_ranks(nproc, argv, port=None, poll_s=0.2):
    """Run `python argv...` as nproc ranks of one job on this node (the
    torch.distributed env contract: RANK, LOCAL_RANK, WORLD_SIZE, MASTER_*).
    The parent only waits: it never initialises the GPU, and the children are
    started as new processes (no exec). If one rank fails the others are
    terminated (a rank blocked in a collective would wait forever). Returns
    the first non-zero exit code, else 0."""
    port = port or free_port()
    procs = []
    for r in range(nproc):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nproc), LOCAL_WORLD_SIZE=str(nproc),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable] + list(argv), env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in live:
                    q.terminate()
        time.sleep(poll_s)
    return rc


# ------------------------------------------------------------ reassembly
class GatherPipeline:
    """Per-step shard production followed by an asynchronous all-gather of the
    shard into the whole vector (the bench step of SURVEY.md 8(e)).

    produce(i, buf) writes step i's shard ([rows, words] int32) into buf.
    With world > 1 the shard and the gathered vector are double-buffered and
    the gather is issued async_op, so step i's all-gather (RCCL's stream)
    overlaps step i+1's kernels; drain() waits for every pending gather.
    collective=True takes the gather path at world 1 too (an initialised
    process group of one rank: bench.py --dist, tests/test_gpu_rccl.py), so
    the RCCL calls of the N-GPU job run on a one-GPU box; the default is
    world > 1.

    proxy_world=P (> world, with the collective): a one-box stand-in for a
    P-rank job's exchange volume and memory. The gathered vectors are sized
    for P ranks, and each step issues a second async all-gather that moves
    the (P - world) / P of the vector the other ranks would send - read from
    the previous step's vector, written into this step's - so every step
    carries the P-rank job's gather bytes and RCCL launches next to the
    kernels (bench.py --proxy-world)."""

    def __init__(self, produce, rows, words, world=1, rank=0, device="cpu", group=None, depth=2, collective=None,
                 proxy_world=None):
        self.produce = produce
        self.world, self.rank, self.group = world, rank, group
        self.rows = rows
        self.coll = world > 1 if collective is None else bool(collective)
        self.nb = depth if self.coll else 1
        self.proxy = proxy_world if (self.coll and proxy_world and proxy_world > world) else None
        vw = self.proxy or world
        self.shards = [torch.empty((rows, words), dtype=torch.int32, device=device) for _ in range(self.nb)]
        self.gathered = ([torch.empty((vw * rows, words), dtype=torch.int32, device=device) for _ in range(self.nb)]
                         if self.coll else None)
        if self.proxy:
            assert self.nb >= 2, "the proxy gather reads the previous step's vector"
            for g in self.gathered:
                g.zero_()
        self.pending = [None] * self.nb

    def step(self, i):
        b = i % self.nb
        for w in self.pending[b] or ():  # the gathers still reading shards[b] must finish first
            w.wait()
        self.pending[b] = None
        buf = self.shards[b]
        self.produce(i, buf)
        if self.coll:
            w = self.world * self.rows
            works = [dist.all_gather_into_tensor(self.gathered[b][:w], buf, group=self.group, async_op=True)]
            if self.proxy:
                # the other ranks' share of the P-rank vector, read from the
                # previous step's vector (its gathers were issued earlier on
                # the same communicator)
                prev = self.gathered[(i - 1) % self.nb]
                per = (self.proxy - self.world) * self.rows // self.world
                works.append(dist.all_gather_into_tensor(self.gathered[b][w:w + per * self.world], prev[:per],
                                                         group=self.group, async_op=True))
            self.pending[b] = works
        return buf

    def drain(self):
        for b in range(self.nb):
            for w in self.pending[b] or ():
                w.wait()
            self.pending[b] = None

    def vector(self, i):
        """The reassembled vector of step i (after drain); the shard itself without a collective."""
        b = i % self.nb
        return self.gathered[b][:self.world * self.rows] if self.coll else self.shards[b]

    def shard(self, i):
        return self.shards[i % self.nb]


def shard_parity(shard, vector, rank, idx, expected):
    """This rank's shard (last step) against expected(i) -> int ciphertext of
    local element i at the sample positions idx, and the shard's copy inside
    the reassembled vector at offset rank * rows (None when world == 1)."""
    from ._native import words_to_ints
    got = words_to_ints(shard[idx].cpu().numpy().view(np.uint32))
    ok = all(expected(int(i)) == g for i, g in zip(idx, got))
    if vector is not None:
        rows = shard.shape[0]
        ok = ok and bool(torch.equal(vector[rank * rows:(rank + 1) * rows], shard))
    return ok


# ------------------------------------------------------------ partial merge
def merge_segment_products(partials, exps, combine, counts=None, group=None, collective=None):
    """Merge every rank's per-segment homomorphic sums (histogram bins).

    partials [nseg, words] int32 and exps [nseg] int32: this rank's segment
    products (an empty segment holds 1 = Enc(0) unobfuscated, exponent 0, the
    reference's fillna(0) + add). They are all-gathered (RCCL on GPU tensors;
    gloo needs CPU tensors, so a gloo group gathers through host memory) and
    each segment's G partials are combined by ONE call
        combine(words [nseg*G, words] segment-major, d [nseg*G] int32,
                seg_begin int64[nseg+1]) -> [nseg, words]
    with d = e - min_g e the alignment of paillier.py:79-86 (xhe_segprod on
    the device: device_combine). counts [nseg] int64 are summed (the
    groupby 'count' column). Returns (words, exponents, counts)."""
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    nseg, words = partials.shape
    coll = world > 1 if collective is None else (bool(collective) and dist.is_initialized())
    if coll:
        dev = partials.device if dist.get_backend(group) == "nccl" else torch.device("cpu")
        allp = torch.empty((world * nseg, words), dtype=torch.int32, device=dev)
        dist.all_gather_into_tensor(allp, partials.to(dev).contiguous(), group=group)
        alle = torch.empty(world * nseg, dtype=torch.int32, device=dev)
        dist.all_gather_into_tensor(alle, exps.to(dev, torch.int32).contiguous(), group=group)
        if counts is not None:
            c = counts.to(dev, torch.int64).clone()
            dist.all_reduce(c, group=group)
            counts = c.to(partials.device)
        allp, alle = allp.to(partials.device), alle.to(partials.device)
    else:
        allp, alle = partials.contiguous(), exps.to(torch.int32)
    seg_major = allp.view(world, nseg, words).transpose(0, 1).reshape(nseg * world, words).contiguous()
    e = alle.view(world, nseg).transpose(0, 1).to(torch.int64)   # [nseg, G]
    emin = e.min(dim=1).values
    d = (e - emin[:, None]).reshape(-1).to(torch.int32).contiguous()
    seg_begin = np.arange(nseg + 1, dtype=np.int64) * world
    out = combine(seg_major, d, seg_begin)
    return out, emin.to(torch.int32), counts


def device_combine(dk, stream=None):
    """combine() for merge_segment_products on the GPU: one xhe_segprod over
    device tensors (include/xhe.h)."""
    import ctypes

    from . import _native as nat

    def combine(words, d, seg_begin):
        nseg = seg_begin.shape[0] - 1
        out = torch.empty((nseg, words.shape[1]), dtype=torch.int32, device=words.device)
        dmax = int(d.max().item()) if d.numel() else 0
        s = stream if stream is not None else torch.cuda.current_stream(words.device).cuda_stream
        nat.check(nat.lib().xhe_segprod(dk.handle, words.data_ptr(), d.data_ptr() if dmax else None, dmax,
                                        words.shape[0], seg_begin.ctypes.data_as(ctypes.c_void_p), nseg,
                                        out.data_ptr(), s), "segprod")
        return out
    return combine
