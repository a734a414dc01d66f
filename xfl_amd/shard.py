"""Element sharding across GPUs of one node.

Encrypt/decrypt/add/scalar-mul are element-independent: rank r owns the
contiguous range [r*ceil(N/G), min(N, (r+1)*ceil(N/G))). The only exchange is
reassembling the ciphertext vector (RCCL all-gather over xGMI; `gloo` on CPU
for tests) and merging per-rank partial products of sums / histograms, which
RCCL cannot reduce (modular product), so partials are all-gathered and
combined locally (the analogue of xgb_actor.merge_hist,
core/tree_ray/xgb_actor.py:447-456).
"""
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
