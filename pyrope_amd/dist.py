"""Multi-GPU orchestration of the sharded scan (one process per GPU, torch.distributed).

Two partitions are implemented:

* LIST-SHARDED (north_star's "IVF lists shard naturally across the GPUs"; the
  default of bench.py since round 5): ListShardedIvf below.  Every rank owns whole lists (a size-balanced
  assignment, list_owners), so each (query, list) pair is scanned by one rank and a rank's per-query work
  shrinks as N grows.

* rows within lists (option ii, rounds 1-4; ShardedIvfStep): the base set is cut into
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


def rank_build_peak_bytes(dim: int, nrows: int, nlist: int, max_list_len: int) -> int:
    """Peak HBM while a rank builds its shard: commit_lists builds the new list store beside the
    old one (2 x the steady-state index bytes) and holds a row-major and a blocked fp32 copy of the rows."""
    ib, _ = rank_memory_plan(dim, nrows, nlist, max_list_len, 1, 1, 1)
    return 2 * ib + 2 * 4 * dim * nrows


# =============================================================================================
# List-sharded IVF_FLAT (C ABI: include/pyrope_ann.h "List-sharded multi-GPU")
# =============================================================================================
SAMPLE_ROWS = 512  # rows of every list replicated for the home rank's threshold (sample16.hip: 16 tiles)


def rank_memory_plan_lists(dim: int, rank_rows: int, nlist: int, max_list_len: int, nq_home: int, world: int,
                           nprobe: int, k: int, fcap: int = 256):
    """(index_bytes, workspace_bytes) of one rank of the list-sharded step (ListShardedIvf), before it
    allocates: its whole lists (rank_rows rows over the global quantizer's nlist lists) plus the replicated
    sample store (min(len, 512) rows of every list, planned as a second index of nlist x 512 rows -- an
    over-estimate: the sample store keeps no row-major copy), and one step's buffers: the search of all
    world x nq_home queries against the rank's lists (pyr_ivf_memory_plan), the plans (home + gathered), the
    records (sent + received), the failure lists and the re-run records."""
    P = min(nprobe, nlist)
    Q = world * nq_home
    ib, wb = rank_memory_plan(dim, rank_rows, nlist, max_list_len, Q, P, k)
    sb, swb = rank_memory_plan(dim, nlist * SAMPLE_ROWS, nlist, SAMPLE_ROWS, nq_home, P, k)
    rb = 16 * (k + 1)
    step = (4 * (2 * P + 1) * (nq_home + Q) + 2 * rb * Q + 4 * world * (1 + fcap) * 2 + 2 * rb * world * fcap
            + 4 * (1 + world) * (1 + nq_home))
    return ib + sb, max(wb, swb) + step


def list_owners(list_len, world: int) -> np.ndarray:
    """Size-balanced owner of every list: lists by length (desc, ties by id) to the rank with the fewest rows
    so far (ties: lowest rank) -- deterministic, so every rank computes the same table."""
    import heapq

    n = len(list_len)
    owner = np.zeros(n, np.int32)
    heap = [(0, r) for r in range(world)]
    for l in sorted(range(n), key=lambda i: (-int(list_len[i]), i)):
        load, r = heapq.heappop(heap)
        owner[l] = r
        heapq.heappush(heap, (load + int(list_len[l]), r))
    return owner


class Comm:
    """The collectives of the list-sharded step over torch.distributed: RCCL ("nccl") works on CUDA tensors,
    gloo on CPU tensors; a tensor on the other side is staged (the one-GPU gloo rehearsal stages CUDA
    tensors through the host, a host-side row exchange under RCCL goes through the GPU).  world == 1:
    plain copies."""

    def __init__(self, world: int):
        self.world = world

    def _dev(self):
        import torch
        import torch.distributed as dist
        if dist.get_backend() == "nccl":
            return torch.device("cuda", torch.cuda.current_device())
        return torch.device("cpu")

    def _run(self, fn, out, *ins):
        d = self._dev()
        o = out if out.device == d else out.to(d)
        i = [t.contiguous() if t.device == d else t.to(d).contiguous() for t in ins]
        fn(o, *i)
        if o is not out:
            out.copy_(o)
        return out

    def all_gather_into(self, out, t):
        """t [rows, ...] of every rank -> out [world * rows, ...] in rank order."""
        import torch.distributed as dist
        if self.world == 1:
            return out.copy_(t)
        if dist.get_backend() == "nccl":
            return self._run(lambda o, i: dist.all_gather_into_tensor(o, i), out, t)
        return self._run(lambda o, i: dist.all_gather(list(o.view((self.world,) + tuple(i.shape)).unbind(0)), i), out, t)

    def all_to_all_single(self, out, t):
        """Equal splits: rows [r * n / world, ...) of t go to rank r; out holds what every rank sent here."""
        import torch.distributed as dist
        if self.world == 1:
            return out.copy_(t)
        return self._run(lambda o, i: dist.all_to_all_single(o, i), out, t)

    def all_reduce_sum(self, t):
        import torch.distributed as dist
        if self.world == 1:
            return t
        return self._run(lambda o, i: (o.copy_(i), dist.all_reduce(o)), t, t)

    def all_to_all_v(self, t, send_counts):
        """Rows of t ([n, ...], grouped by destination rank, send_counts[r] rows to rank r) -> the rows every
        rank sent here, in source-rank order, and their counts."""
        import torch
        import torch.distributed as dist
        if self.world == 1:
            return t.clone(), list(send_counts)
        sc = torch.tensor(send_counts, dtype=torch.int64)
        rc = torch.empty_like(sc)
        self._run(lambda o, i: dist.all_to_all_single(o, i), rc, sc)
        out = torch.empty((int(rc.sum()),) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        self._run(lambda o, i: dist.all_to_all_single(o, i, output_split_sizes=rc.tolist(),
                                                      input_split_sizes=sc.tolist()), out, t)
        return out, rc.tolist()

    def max_int(self, v: int, rank: int) -> int:
        import torch
        t = torch.zeros(self.world, dtype=torch.int64)
        t[rank] = int(v)
        return int(self.all_reduce_sum(t).max())


def shard_plan_stride(width: int, budget: bool) -> int:
    """int32 row stride of a list-sharded plan (pyr_shard_plan_stride): P probes + T_q, and with a MaxScans
    budget the P remaining budgets."""
    return width + 1 + (width if budget else 0)


class DeviceShardEngine:
    """The list-sharded step's per-rank operations on libpyrope_hip (IVF_FLAT shard index, device buffers
    as torch tensors, one stream)."""

    def __init__(self, index, k: int, options=None, stream=None):
        self.index, self.k, self.options, self._stream = index, k, options, stream

    @property
    def budget(self) -> bool:
        """A MaxScans search: the plans carry the budget left at every probe (IvfFlatVectorIndex.cs:202-212)."""
        return self.options is not None and getattr(self.options, "max_scans", None) is not None

    @property
    def stream(self) -> int:
        """The given stream, else torch's current stream at the time of the call (so a phase captured
        under torch.cuda.graph enqueues on the capture stream)."""
        if self._stream is not None:
            return self._stream
        import torch
        return torch.cuda.current_stream().cuda_stream

    def prepare(self, q_home, plan):
        return self.index.shard_prepare_device(q_home.data_ptr(), q_home.shape[0], self.k, plan.data_ptr(),
                                               self.stream, self.options)

    def search(self, q_all, plan_all, width, rec):
        self.index.shard_search_device(q_all.data_ptr(), q_all.shape[0], self.k, plan_all.data_ptr(), width,
                                       rec.data_ptr(), self.stream, budgets=self.budget)

    def merge(self, rec_parts, out_s, out_l, fail):
        from . import _lib
        world, n = rec_parts.shape[0], rec_parts.shape[1]
        _lib.check(_lib.load().pyr_shard_merge_device(rec_parts.data_ptr(), world, n, self.k, None, 0,
                                                      out_s.data_ptr(), out_l.data_ptr(), None, fail.data_ptr(),
                                                      fail.shape[0] - 1, self.stream))

    def rerun(self, q_all, plan_all, width, fails_all, nq_home, rec):
        world, f1 = fails_all.shape
        self.index.shard_rerun_device(q_all.data_ptr(), q_all.shape[0], self.k, plan_all.data_ptr(), width,
                                      fails_all.data_ptr(), world, f1 - 1, nq_home, rec.data_ptr(), self.stream,
                                      budgets=self.budget)

    def merge_rerun(self, rec_parts, fail_home, out_s, out_l):
        from . import _lib
        world, fcap = rec_parts.shape[0], rec_parts.shape[1]
        _lib.check(_lib.load().pyr_shard_merge_device(rec_parts.data_ptr(), world, fcap, self.k, fail_home.data_ptr(),
                                                      fcap, out_s.data_ptr(), out_l.data_ptr(), None, None, 0,
                                                      self.stream))


class ListShardedIvf:
    """One list-sharded multi-GPU IVF_FLAT search step (include/pyrope_ann.h "List-sharded multi-GPU"):

      1. plan: the home rank ranks the quantizer for its nq_local queries and takes T_q from its replicated
         sample of every list (engine.prepare); with a MaxScans budget the plan also carries, per probe, the
         budget left when that list is reached (IvfFlatVectorIndex.cs:202-212);
      2. all_gather(plans): every rank gets every query's probe lists and threshold;
      3. every rank scans the (query, list) pairs of the lists it owns -> one record per query (exact local
         top-k + the bound of the rows it left out; engine.search);
      4. all_to_all(records): each home receives its queries' records from every rank;
      5. the home merges and certifies (k-th merged score > every rank's bound; engine.merge); its fail list
         keeps EVERY failing query (it is sized to the home's batch);
      6. all_gather(the first fcap entries of every fail list) [world][1 + fcap];
      7. every rank runs the exact scan of those failures over its lists (engine.rerun);
      8. all_to_all(re-run records) and the home merges them into its results (engine.merge_rerun).

    The failure counts of every home arrive with step 6 on every rank; the host reads them (an event on that
    copy) and every rank makes the same decision: no failure anywhere (the usual step) -- steps 7-8 are
    skipped; else steps 7-8 for the first fcap failures of every home, and when a home has more than fcap,
    further rounds: one all_gather of the whole fail lists, then per round of fcap entries steps 7-8 again.
    So every failing query is re-run exactly, whatever the data.  `stats` holds the last
    step's largest failure count and its extra rounds.  All buffers are allocated once (torch tensors on
    `device`); the step is a generator of collectives (_ops), which __call__ runs over `comm` and
    LocalShardGroup runs for W ranks in one process.
    """

    def __init__(self, engine, comm, nq_local: int, k: int, width: int, rank: int, world: int, device=None,
                 fcap: int = 256):
        import torch

        self.engine, self.comm = engine, comm
        self.nq, self.k, self.width, self.rank, self.world = nq_local, k, width, rank, world
        self.fcap = max(1, min(int(fcap), nq_local)) if nq_local > 0 else max(1, int(fcap))
        fcap = self.fcap
        self.budget = bool(getattr(engine, "budget", False))
        S = shard_plan_stride(width, self.budget)
        rb = 16 * (k + 1)
        Q = nq_local * world
        self.plan_home = torch.empty((nq_local, S), dtype=torch.int32, device=device)
        self.plan_all = torch.empty((Q, S), dtype=torch.int32, device=device)
        self.rec = torch.empty((Q, rb), dtype=torch.uint8, device=device)
        self.rec_home = torch.empty((world, nq_local, rb), dtype=torch.uint8, device=device)
        self.fail_home = torch.zeros((1 + nq_local,), dtype=torch.int32, device=device)
        self.fail_all = torch.zeros((world, 1 + fcap), dtype=torch.int32, device=device)
        self.fail_full = None  # [world][1 + nq_local], allocated by the first step that needs a second round
        self.fail_round = torch.zeros((world, 1 + fcap), dtype=torch.int32, device=device)
        self.rrec = torch.zeros((world * fcap, rb), dtype=torch.uint8, device=device)
        self.rrec_home = torch.zeros((world, fcap, rb), dtype=torch.uint8, device=device)
        self.out_s = torch.empty((nq_local, k), dtype=torch.float32, device=device)
        self.out_l = torch.empty((nq_local, k), dtype=torch.int64, device=device)
        cuda = self.fail_all.is_cuda
        self._counts = torch.zeros((world,), dtype=torch.int32, pin_memory=cuda)
        self._counts_ev = torch.cuda.Event() if cuda else None
        self.stats = {"max_failures": 0, "extra_rounds": 0}
        self.max_fail = 0        # the most failures of one home in any step so far
        self.timing = False
        self.collective_ms = {}

    def _timed(self, name, fn):
        return ShardedIvfStep._timed(self, name, fn)

    @property
    def probes_all(self):  # ShardedIvfStep._timed checks .is_cuda on it
        return self.plan_all

    # the device work between two collectives (each may be replayed from a hipGraph: capture())
    def _phase(self, name, q_all):
        g = getattr(self, "graphs", {}).get(name)
        if g is not None:
            g.replay()
            return
        nq, r, e, P = self.nq, self.rank, self.engine, self.width
        if name == "prepare":
            got = e.prepare(q_all[r * nq:(r + 1) * nq], self.plan_home)
            if got != P:
                raise ValueError(f"plan width {got} != {P}")
        elif name == "search":
            e.search(q_all, self.plan_all, P, self.rec)
        elif name == "merge":
            e.merge(self.rec_home, self.out_s, self.out_l, self.fail_home)
        elif name == "rerun":
            e.rerun(q_all, self.plan_all, P, self.fail_all, nq, self.rrec)
        else:  # "finish"
            e.merge_rerun(self.rrec_home, self.fail_home, self.out_s, self.out_l)

    PHASES = ("prepare", "search", "merge", "rerun", "finish")

    def capture(self, q_all):
        """Capture the five device phases into hipGraphs (the collectives stay outside them), replayed by
        every later call on the same q_all buffer.  One plain step on the capture stream sizes its
        workspaces first (no allocation inside a capture).  Overflow rounds run uncaptured."""
        import torch
        gst = torch.cuda.Stream()
        gst.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(gst):
            self(q_all)
            # (a step without failures skips the re-run: its phases size their workspaces here, on the last
            # step's fail lists)
            self._phase("rerun", q_all)
            self._phase("finish", q_all)
        gst.synchronize()
        graphs = {}
        for name in self.PHASES:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=gst):
                self._phase(name, q_all)
            graphs[name] = g
        torch.cuda.synchronize()
        self.graphs = graphs

    def _read_counts(self):
        """Every home's failure count (fail_all[:, 0], the same on every rank) -> numpy; the device copy was
        enqueued after the fail-list gather (_note_counts), so this waits for that point of the step only."""
        if self._counts_ev is not None:
            self._counts_ev.synchronize()
        return self._counts.numpy().copy()

    def _note_counts(self):
        if self._counts_ev is not None:
            self._counts.copy_(self.fail_all[:, 0], non_blocking=True)
            self._counts_ev.record()
        else:
            self._counts.copy_(self.fail_all[:, 0])

    def _ops(self, q_all):
        """The step as a generator: device phases run inline; each collective is yielded as
        (kind, out, in, name) with kind "gather" (all_gather_into) or "a2a" (equal-split all_to_all) for the
        caller to perform before resuming."""
        nq, w, fcap = self.nq, self.world, self.fcap
        self._phase("prepare", q_all)
        yield ("gather", self.plan_all, self.plan_home, "plan_allgather")
        self._phase("search", q_all)
        yield ("a2a", self.rec_home.view(w * nq, -1), self.rec, "record_alltoall")
        self._phase("merge", q_all)
        yield ("gather", self.fail_all, self.fail_home[:1 + fcap], "fail_allgather")
        # every home's failure count, the same on every rank: with none anywhere (the usual step) the re-run's
        # phases and its all_to_all are skipped; else rounds of fcap failures per home
        self._note_counts()
        counts = self._read_counts()
        mx = int(counts.max()) if len(counts) else 0
        extra = max(0, (mx - 1) // fcap) if mx > fcap else 0
        self.stats = {"max_failures": mx, "extra_rounds": extra}
        self.max_fail = max(self.max_fail, mx)
        if mx == 0:
            return
        self._phase("rerun", q_all)
        yield ("a2a", self.rrec_home.view(w * fcap, -1), self.rrec, "rerun_alltoall")
        self._phase("finish", q_all)
        if extra == 0:
            return
        import torch
        if self.fail_full is None:
            self.fail_full = torch.zeros((w, 1 + nq), dtype=torch.int32, device=self.fail_home.device)
        yield ("gather", self.fail_full, self.fail_home, "fail_full_allgather")
        ct = torch.as_tensor(counts, dtype=torch.int32, device=self.fail_home.device)
        for j in range(1, extra + 1):
            off = j * fcap
            # round j: entries [off, off + fcap) of every home's fail list, in the [1 + fcap] form
            self.fail_round.zero_()
            self.fail_round[:, 0] = torch.clamp(ct - off, 0, fcap)
            m = min(fcap, nq - off)
            if m > 0:
                self.fail_round[:, 1:1 + m] = self.fail_full[:, 1 + off:1 + off + m]
            self.engine.rerun(q_all, self.plan_all, self.width, self.fail_round, nq, self.rrec)
            yield ("a2a", self.rrec_home.view(w * fcap, -1), self.rrec, "rerun_alltoall")
            self.engine.merge_rerun(self.rrec_home, self.fail_round[self.rank], self.out_s, self.out_l)

    def __call__(self, q_all):
        c = self.comm
        for kind, out, inp, name in self._ops(q_all):
            if kind == "gather":
                self._timed(name, lambda: c.all_gather_into(out, inp))
            else:
                self._timed(name, lambda: c.all_to_all_single(out, inp))
        return self.out_s, self.out_l


class LocalShardGroup:
    """W ranks of the list-sharded step driven from one process (tests, scripts/rank_shape.py): the steps'
    generators (ListShardedIvf._ops) advance in lockstep and each collective is done as device copies
    between the ranks' buffers -- the same orchestration bench.py runs over RCCL, collectives aside."""

    def __init__(self, steps):
        self.steps = list(steps)

    def __call__(self, q_all):
        W = len(self.steps)
        gens = [s._ops(q_all) for s in self.steps]
        while True:
            ops = [next(g, None) for g in gens]
            if all(o is None for o in ops):
                break
            if any(o is None for o in ops) or len({(o[0], o[3]) for o in ops}) != 1:
                raise RuntimeError("list-sharded ranks diverged: " + repr([o and o[3] for o in ops]))
            kind = ops[0][0]
            for r, (_, out, _, _) in enumerate(ops):
                ov = out.view(W, -1)
                for s in range(W):
                    src = ops[s][2]
                    ov[s].copy_(src.reshape(-1) if kind == "gather" else src.reshape(W, -1)[r])
        return [(s.out_s, s.out_l) for s in self.steps]


def exchange_rows(comm, rank: int, world: int, chunks, centroids, metric, owner_of=None, device: int = 0,
                  add=None, assign_fn=None):
    """Give every rank its WHOLE lists.

    chunks(): iterator over this rank's (labels, rows) in label order, the same number of calls on every rank
    per round (bench.py shard_chunks: round i of every rank covers one contiguous range of generator blocks).
    Pass 1 assigns every row to its list (KMeansUtils.FindNearestCentroid, assign_fn) and sums the list
    lengths over the ranks; owners come from list_owners unless owner_of is given.  Pass 2 sends each row to
    its list's owner (all_to_all_v) round by round; the receiver sorts a round by label, so every list gets
    its rows in label order -- the unsharded index's list order -- and hands them to add(labels, rows).
    The first SAMPLE_ROWS rows of each owned list are kept for the replicated sample.

    Returns (list_len [nlist] int64, owner [nlist] int32, samples {list: rows}) of this rank."""
    import torch

    if assign_fn is None:
        from .vector import assign as assign_fn_dev

        def assign_fn(c, x):
            return assign_fn_dev(c, x, metric, device)
    nl = centroids.shape[0]
    counts = np.zeros(nl, np.int64)
    asg_rounds = []
    for labs, x in chunks():
        a = assign_fn(centroids, x)
        asg_rounds.append(a)
        counts += np.bincount(a, minlength=nl)
    rounds = comm.max_int(len(asg_rounds), rank)  # a rank with fewer rounds sends nothing in the last ones
    glen_t = torch.from_numpy(counts.copy())
    comm.all_reduce_sum(glen_t)
    glen = glen_t.numpy().astype(np.int64)
    owner = list_owners(glen, world) if owner_of is None else np.asarray(owner_of, np.int32)
    samples = {}
    dim = centroids.shape[1]

    def padded():
        yield from zip(chunks(), asg_rounds)
        for _ in range(rounds - len(asg_rounds)):
            yield (np.zeros(0, np.int64), np.zeros((0, dim), np.float32)), np.zeros(0, np.int32)

    for (labs, x), a in padded():
        dst = owner[a]
        order = np.argsort(dst, kind="stable")
        send = np.bincount(dst, minlength=world).tolist()
        payload = np.concatenate([x[order], labs[order].astype(np.int64).view(np.float32).reshape(-1, 2),
                                  a[order].astype(np.int32).view(np.float32).reshape(-1, 1)], axis=1)
        got, _ = comm.all_to_all_v(torch.from_numpy(np.ascontiguousarray(payload)), send)
        got = got.numpy()
        d = x.shape[1]
        rl = np.ascontiguousarray(got[:, d:d + 2]).view(np.int64).reshape(-1)
        ra = np.ascontiguousarray(got[:, d + 2:d + 3]).view(np.int32).reshape(-1)
        o = np.argsort(rl, kind="stable")
        rl, ra, rx = rl[o], ra[o], np.ascontiguousarray(got[o, :d])
        if add is not None and len(rl):
            add(rl, rx)
        for li in np.unique(ra):
            have = samples.get(int(li))
            n0 = 0 if have is None else len(have)
            if n0 >= SAMPLE_ROWS:
                continue
            rows = rx[ra == li][:SAMPLE_ROWS - n0]
            samples[int(li)] = rows if have is None else np.concatenate([have, rows])
    return glen, owner, samples


def gather_samples(comm, rank: int, world: int, glen, owner, samples, dim: int):
    """All ranks' owned-list samples -> (rows [sum counts, dim] in list order, counts [nlist]) everywhere."""
    import torch

    nl = len(glen)
    mine = [l for l in range(nl) if owner[l] == rank]
    block = np.concatenate([samples.get(l, np.zeros((0, dim), np.float32)) for l in mine]) if mine else \
        np.zeros((0, dim), np.float32)
    n_t = torch.tensor([block.shape[0]], dtype=torch.int64)
    sizes = torch.zeros(world, dtype=torch.int64)
    sizes[rank] = n_t[0]
    comm.all_reduce_sum(sizes)
    smax = int(sizes.max())
    pad = np.zeros((max(smax, 1), dim), np.float32)
    pad[:block.shape[0]] = block
    allb = torch.empty((world, max(smax, 1), dim), dtype=torch.float32)
    comm.all_gather_into(allb.view(world * max(smax, 1), dim), torch.from_numpy(pad))
    allb = allb.numpy()
    counts = np.minimum(np.asarray(glen, np.int64), SAMPLE_ROWS)
    pos = np.zeros(world, np.int64)
    out = []
    for l in range(nl):  # each rank's block holds its owned lists in id order
        o = int(owner[l])
        out.append(allb[o, pos[o]:pos[o] + counts[l]])
        pos[o] += counts[l]
    return (np.concatenate(out) if out else np.zeros((0, dim), np.float32)), counts
