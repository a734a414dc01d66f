"""The RCCL (torch.distributed "nccl") code path of the multi-GPU job, run on
one GPU as a process group of one rank.

bench.py --gpus N and BASELINE configs 4/5 move device tensors through RCCL:
the async all-gather of ciphertext shards (shard.GatherPipeline, SURVEY.md
8(e); the reference's process-pool split, paillier.py:321-332) and the
all-gather + all-reduce of per-rank partial histograms
(shard.merge_segment_products, the analogue of xgb_actor.py:447-456
merge_hist). At world 1 those calls are skipped by default, so here they are
forced (collective=True) inside a fresh child process that creates a real
RCCL communicator with the same init_process_group call as bench.py:

* 3 GatherPipeline steps of the bench's own encrypt step on the 3072-bit
  fixture key (device encode + ChaCha draws + DJN-CRT encrypt), gathered
  async_op on device tensors; the gathered vector equals the oracle;
* merge_segment_products through its nccl branch with the device combine
  (xhe_segprod) on the golden ops.hist: equal to the reference's groupby sum;
* the bench's timing reduction (all_reduce MAX of a float64) and barrier;

and bench.py --gpus 1 --dist end to end (the same flow as an N-rank run)."""
import json
import os
import subprocess
import sys

import pytest

from tests.conftest import ROOT

pytestmark = pytest.mark.gpu


def _rccl_child(q):
    sys.path.insert(0, ROOT)
    try:
        import numpy as np
        import torch
        import torch.distributed as dist

        from oracle import paillier_oracle as O
        from tests.conftest import FIXTURES, load_fixture
        from tests.test_gpu_gather import ROWS, SAMPLE, _Encryptor, _expected, _ints, _key
        from tests.test_gpu_shard import _case, _dkey, _local_partials_device
        from xfl_amd import _native as nat
        from xfl_amd.shard import GatherPipeline, device_combine, free_port, merge_segment_products, shard_parity

        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(free_port())
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
        res = {"backend": dist.get_backend()}

        # ---- reassembly: async all-gather of device shards
        dk, (p, q_, h) = _key()
        okey = O.derive_private(p, q_, h)
        enc = _Encryptor(dk, 0)
        pipe = GatherPipeline(enc, ROWS, dk.n2w, world=1, rank=0, device="cuda", collective=True)
        for i in range(3):  # the double buffer wraps around
            pipe.step(i)
        pipe.drain()
        torch.cuda.synchronize()
        last = 2
        vec = pipe.vector(last)
        res["gather_is_separate_buffer"] = vec.data_ptr() != pipe.shard(last).data_ptr()
        res["gather_on_device"] = vec.device.type == "cuda"
        draws = enc.draws(last)
        res["gather_oracle"] = _ints(vec[list(SAMPLE)]) == [_expected(okey, enc, last, i, draws) for i in SAMPLE]
        res["gather_parity"] = shard_parity(pipe.shard(last), vec, 0, [0, ROWS - 1],
                                            lambda i: _expected(okey, enc, last, i, draws))
        # step 1's gathered buffer holds step 1's ciphertexts, not step 2's
        d1 = enc.draws(1)
        res["gather_step1"] = _ints(pipe.vector(1)[[0]]) == [_expected(okey, enc, 1, 0, d1)]

        # ---- partial-histogram merge through the nccl branch
        g = load_fixture(FIXTURES[0])
        hk = _dkey(g)
        raws, exps, bins, nb, want = _case(g)
        parts, pe, cnt = _local_partials_device(hk, raws, exps, bins, nb)
        out, eout, counts = merge_segment_products(parts, pe, device_combine(hk), counts=cnt, collective=True)
        torch.cuda.synchronize()
        res["merge_on_device"] = out.device.type == "cuda" and counts.device.type == "cuda"
        res["merge_golden"] = (nat.words_to_ints(out.cpu().numpy().view(np.uint32)), eout.tolist(),
                               counts.tolist()) == want

        # ---- bench.py's timing reduction
        t = torch.tensor([1.25], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.barrier()
        res["allreduce"] = float(t.item()) == 1.25
        dist.destroy_process_group()
        q.put(res)
    except Exception as exc:  # noqa: BLE001 - reported to the parent instead of hanging it
        import traceback
        q.put({"error": repr(exc), "tb": traceback.format_exc()})


def test_rccl_world1_gather_merge_and_reduce():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_child, args=(q,))
    p.start()
    try:
        res = q.get(timeout=240)
    finally:
        p.join(timeout=60)
        if p.is_alive():
            p.kill()
    assert "error" not in res, res.get("tb", res)
    assert res.pop("backend") == "nccl"
    assert all(res.values()), res


def test_bench_dist_world1():
    """bench.py --gpus 1 --dist: init_process_group, async all-gather of every
    step, barriers and the max-over-ranks all-reduce of an N-rank run."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--dist", "--n", "8192", "--steps", "3",
           "--warmup", "1", "--win", "12", "--no-ops", "--no-cpu-baseline"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    rec = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert rec["parity_sample_ok"] is True
    assert rec["config"]["parallelism"] == "shard1+rccl"
    assert rec["n_gpus"] == 1 and rec["value"] > 0
    assert rec["roofline"]["kernel"] == "k_djn_pmd"
