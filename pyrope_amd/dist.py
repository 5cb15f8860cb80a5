"""Multi-GPU orchestration of the sharded scan (one process per GPU, torch.distributed).

Sharding (option ii "rows within lists"): the base set is cut into
generator blocks of BLOCK_ROWS rows and rank r holds every block b with b % world == r
(shard_blocks).  Every rank builds its shard with the SAME coarse quantizer (trained once
and broadcast), so each rank's lists are row subsets of the unsharded lists, in the same
relative order.

One step of the batched search (sharded_ivf_step, what bench.py times):
  1. each rank ranks the coarse quantizer for its own slice of the batch (probe),
  2. one all_gather assembles every query's probe lists,
  3. each rank scans its shard of those lists for the whole batch (search) -> partial top-k,
  4. one all_gather of the partials (b x k x (4 + 8) bytes per rank) and a merge by
     (score desc, label asc) give the global top-k.
These two all_gathers are the only collectives on the data path.  On GPUs they are RCCL
(backend "nccl") over xGMI and the merge is libpyrope_hip's pyr_merge_topk_device; the same
function runs on CPU with gloo and the oracle as the scan (tests/test_dist.py).
"""
from __future__ import annotations

from typing import Callable, List, Tuple

import numpy as np

BLOCK_ROWS = 65536  # == vector.BLOCK_ROWS: generator blocks are the sharding unit


def shard_blocks(n: int, world: int, rank: int, block_rows: int = BLOCK_ROWS) -> List[Tuple[int, int]]:
    """Row ranges [a, b) of the blocks owned by `rank`: block i (rows i*block_rows ..) iff i % world == rank."""
    nb = (n + block_rows - 1) // block_rows
    return [(b * block_rows, min(n, (b + 1) * block_rows)) for b in range(rank, nb, world)]


def shard_labels(n: int, world: int, rank: int, block_rows: int = BLOCK_ROWS) -> np.ndarray:
    """Base rows (= labels) owned by `rank`, in base-row order."""
    parts = [np.arange(a, b, dtype=np.int64) for a, b in shard_blocks(n, world, rank, block_rows)]
    return np.concatenate(parts) if parts else np.zeros(0, np.int64)


def all_gather_rows(t, world: int):
    """[rows, ...] per rank -> [world * rows, ...] in rank order (nccl: one all_gather_into_tensor)."""
    import torch
    import torch.distributed as dist

    if world == 1:
        return t
    t = t.contiguous()
    if dist.get_backend() == "nccl":
        out = torch.empty((world * t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        dist.all_gather_into_tensor(out, t)
        return out
    parts = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(parts, t)
    return torch.cat(parts)


def gather_partials(scores, labels, world: int):
    """All-gather per-rank partial (scores [Q,k] fp32, labels [Q,k] int64) -> [Q, world, k] each."""
    if world == 1:
        return scores.unsqueeze(1), labels.unsqueeze(1)
    Q, k = scores.shape
    s_all = all_gather_rows(scores, world).reshape(world, Q, k)
    l_all = all_gather_rows(labels, world).reshape(world, Q, k)
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


def sharded_ivf_step(queries, nq_local: int, rank: int, world: int, probe: Callable, search: Callable,
                     merge: Callable, k: int):
    """One batched multi-GPU IVF search step (module docstring).

    queries: [world * nq_local, D], identical on every rank; rank r owns rows
    [r * nq_local, (r + 1) * nq_local) for the coarse ranking.
    probe(q_slice) -> int32 probe lists [nq_local, P]
    search(queries, probes_all) -> (scores [Q, k], labels [Q, k]) over this rank's shard
    merge(s_parts [Q, world, k], l_parts [Q, world, k], k) -> (scores [Q, k], labels [Q, k])
    """
    mine = queries[rank * nq_local:(rank + 1) * nq_local]
    probes_all = all_gather_rows(probe(mine), world)
    s, lab = search(queries, probes_all)
    if world == 1:
        return s, lab
    sp, lp = gather_partials(s, lab, world)
    return merge(sp, lp, k)


def sharded_search(local_search: Callable, merge: Callable, queries, k: int, world: int):
    """local_search(queries, k) -> (scores, labels) on this rank's shard; then gather + merge."""
    s, l = local_search(queries, k)
    if world == 1:
        return s, l
    s_parts, l_parts = gather_partials(s, l, world)
    return merge(s_parts, l_parts, k)
