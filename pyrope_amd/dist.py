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

    if world == 1:
        return t
    t = t.contiguous()
    out = torch.empty((world * t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    return all_gather_into(out, t, world)


def all_gather_into(out, t, world: int):
    """All-gather t ([rows, ...] on every rank) into the preallocated out ([world * rows, ...], rank
    order): nccl (RCCL) writes it with one all_gather_into_tensor, gloo through per-rank views of it."""
    import torch.distributed as dist

    if world == 1:
        out.copy_(t)
        return out
    t = t.contiguous()
    if dist.get_backend() == "nccl":
        dist.all_gather_into_tensor(out, t)
    else:
        dist.all_gather(list(out.chunk(world)), t)
    return out


def gather_partials(scores, labels, world: int):
    """All-gather per-rank partial (scores [Q,k] fp32, labels [Q,k] int64) -> [Q, world, k] each."""
    if world == 1:
        return scores.unsqueeze(1), labels.unsqueeze(1)
    Q, k = scores.shape
    s_all = all_gather_rows(scores, world).reshape(world, Q, k)
    l_all = all_gather_rows(labels, world).reshape(world, Q, k)
    return s_all.transpose(0, 1).contiguous(), l_all.transpose(0, 1).contiguous()


def merge_device(s_parts, l_parts, k: int, stream: int = 0, part_major: bool = False) -> Tuple[object, object]:
    """On-device merge of partial lists with pyr_merge_topk_parts_device: [Q, parts, k] each, or
    [parts, Q, k] (part_major, the layout an all_gather leaves)."""
    import torch

    from . import _lib
    L = _lib.load()
    if part_major:
        parts, Q, _ = s_parts.shape
    else:
        Q, parts, _ = s_parts.shape
    s_out = torch.empty((Q, k), dtype=torch.float32, device=s_parts.device)
    l_out = torch.empty((Q, k), dtype=torch.int64, device=s_parts.device)
    _lib.check(L.pyr_merge_topk_parts_device(s_parts.data_ptr(), l_parts.data_ptr(), Q, parts, k, int(part_major),
                                             s_out.data_ptr(), l_out.data_ptr(), stream))
    return s_out, l_out


class ShardedIvfStep:
    """One batched multi-GPU IVF search step (module docstring) over buffers allocated once.

    nq_local queries per rank, `width` probes per query, top-k; the probe lists of all ranks
    ([world * nq_local, width] int32) and the all-gathered partials ([world, Q, k] fp32 / int64, rank
    major: merged as they land, no transpose) live for the whole run.
      probe(q_slice) -> int32 probe lists [nq_local, width]
      search(queries, probes_all) -> (scores [Q, k], labels [Q, k]) over this rank's shard
      merge(s_all [world, Q, k], l_all [world, Q, k], k) -> (scores [Q, k], labels [Q, k])
    With timing on, the two collectives are timed (CUDA events on the current stream; wall clock on
    CPU) into `collective_ms` = {"probe_allgather": ms, "partial_allgather": ms} of the last call.
    """

    def __init__(self, nq_local: int, width: int, k: int, rank: int, world: int, device=None):
        import torch

        self.nq_local, self.width, self.k, self.rank, self.world = nq_local, width, k, rank, world
        Q = nq_local * world
        self.probes_all = torch.empty((Q, width), dtype=torch.int32, device=device)
        self.s_all = torch.empty((world, Q, k), dtype=torch.float32, device=device)
        self.l_all = torch.empty((world, Q, k), dtype=torch.int64, device=device)
        self.timing = False
        self.collective_ms = {}

    def _timed(self, name, fn):
        if not self.timing:
            return fn()
        import time

        import torch
        if self.probes_all.is_cuda:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            r = fn()
            b.record()
            b.synchronize()
            self.collective_ms[name] = a.elapsed_time(b)
        else:
            t = time.perf_counter()
            r = fn()
            self.collective_ms[name] = (time.perf_counter() - t) * 1e3
        return r

    def __call__(self, queries, probe: Callable, search: Callable, merge: Callable):
        nq, w, r, k = self.nq_local, self.world, self.rank, self.k
        mine = queries[r * nq:(r + 1) * nq]
        p = probe(mine)
        if w == 1:
            return search(queries, p)
        self._timed("probe_allgather", lambda: all_gather_into(self.probes_all, p, w))
        s, lab = search(queries, self.probes_all)
        Q = nq * w
        self._timed("partial_allgather", lambda: (all_gather_into(self.s_all.view(w * Q, k), s, w),
                                                  all_gather_into(self.l_all.view(w * Q, k), lab, w)))
        return merge(self.s_all, self.l_all, k)


def sharded_ivf_step(queries, nq_local: int, rank: int, world: int, probe: Callable, search: Callable,
                     merge: Callable, k: int):
    """One step over freshly allocated buffers (ShardedIvfStep; merge takes [world, Q, k])."""
    width = None

    def probe_w(qs):
        nonlocal width
        p = probe(qs)
        width = p.shape[1]
        return p

    mine = queries[rank * nq_local:(rank + 1) * nq_local]
    p = probe_w(mine)
    step = ShardedIvfStep(nq_local, width, k, rank, world, device=p.device)
    return step(queries, lambda _: p, search, merge)


def sharded_search(local_search: Callable, merge: Callable, queries, k: int, world: int):
    """local_search(queries, k) -> (scores, labels) on this rank's shard; then gather + merge."""
    s, l = local_search(queries, k)
    if world == 1:
        return s, l
    s_parts, l_parts = gather_partials(s, l, world)
    return merge(s_parts, l_parts, k)


def rank_memory_plan(dim: int, nrows: int, nlist: int, max_list_len: int, nq: int, nprobe: int, k: int):
    """(index_bytes, workspace_bytes) of one rank: its IVF_FLAT shard and one batched search of nq
    queries (pyr_ivf_memory_plan; host arithmetic, no GPU needed)."""
    import ctypes as C

    from . import _lib
    L = _lib.load()
    ib, wb = C.c_int64(), C.c_int64()
    _lib.check(L.pyr_ivf_memory_plan(dim, nrows, nlist, max_list_len, nq, nprobe, k, C.byref(ib), C.byref(wb)))
    return ib.value, wb.value
