"""Multi-GPU orchestration of the sharded scan (one process per GPU, torch.distributed).

Sharding (option ii "rows within lists"): rank r holds base row i
iff i % world == r, and every rank builds its shard with the SAME coarse
quantizer (trained once, reference-identical, on the full data).  Every rank
scans its shard for the whole query batch; the per-rank partial top-k lists
(score desc, label asc) are exchanged with one all_gather and merged, ties by
label ascending -- which equals the unsharded index's storage order because
labels are assigned in base-row order.

The exchange is the only collective on the data path.  On GPUs it is RCCL
(backend "nccl") over xGMI and the merge is libpyrope_hip's
pyr_merge_topk_device; the same orchestration runs on CPU with gloo for tests.
"""
from __future__ import annotations

from typing import Callable, Tuple

import numpy as np


def shard_labels(n: int, world: int, rank: int) -> np.ndarray:
    """Base rows (= labels) owned by `rank`: i % world == rank, in base-row order."""
    return np.arange(rank, n, world, dtype=np.int64)


def gather_partials(scores, labels, world: int):
    """All-gather per-rank partial (scores [Q,k] fp32, labels [Q,k] int64) -> [Q, world, k] each."""
    import torch
    import torch.distributed as dist

    if world == 1:
        return scores.unsqueeze(1), labels.unsqueeze(1)
    if dist.get_backend() == "nccl":
        s_all = torch.empty((world,) + tuple(scores.shape), dtype=scores.dtype, device=scores.device)
        l_all = torch.empty((world,) + tuple(labels.shape), dtype=labels.dtype, device=labels.device)
        dist.all_gather_into_tensor(s_all, scores.contiguous())
        dist.all_gather_into_tensor(l_all, labels.contiguous())
    else:
        s_list = [torch.empty_like(scores) for _ in range(world)]
        l_list = [torch.empty_like(labels) for _ in range(world)]
        dist.all_gather(s_list, scores.contiguous())
        dist.all_gather(l_list, labels.contiguous())
        s_all, l_all = torch.stack(s_list), torch.stack(l_list)
    return s_all.transpose(0, 1).contiguous(), l_all.transpose(0, 1).contiguous()


def merge_device(s_parts, l_parts, k: int, stream: int = 0) -> Tuple[object, object]:
    """On-device merge of [Q, parts, k] partial lists with pyr_merge_topk_device."""
    import torch

    from . import _lib
    L = _lib.load()
    Q, parts, _ = s_parts.shape
    s_out = torch.empty((Q, k), dtype=torch.float32, device=s_parts.device)
    l_out = torch.empty((Q, k), dtype=torch.int64, device=s_parts.device)
    _lib.check(L.pyr_merge_topk_device(s_parts.data_ptr(), l_parts.data_ptr(), Q, parts, k, s_out.data_ptr(),
                                       l_out.data_ptr(), stream))
    return s_out, l_out


def sharded_search(local_search: Callable, merge: Callable, queries, k: int, world: int):
    """local_search(queries, k) -> (scores, labels) on this rank's shard; then gather + merge."""
    s, l = local_search(queries, k)
    if world == 1:
        return s, l
    s_parts, l_parts = gather_partials(s, l, world)
    return merge(s_parts, l_parts, k)
