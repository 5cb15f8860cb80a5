#!/usr/bin/env python3
"""bench.py -- QPS + recall@10 of the IVF_FLAT scan on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[2], I1): IVF_FLAT d=128, N=10M base vectors, nlist=1024,
nprobe=32, top-10, synthetic uniform [0,1) vectors from the reference benchmark's generator
(Pyrope.Benchmarks/Program.cs:251-263) in row blocks of 65,536 rows (block b = Random(42 + b),
SURVEY.md 8(d)'s large-N deviation; queries = Random(1337)).  `--n 80000000 --nlist 8192`
is configs[4] (M8).

A step = one batched search of 10,000 queries per GPU, queries and results resident in HBM.

--gpus N: one process per GPU.  Launched by torch.distributed.run (RANK/WORLD_SIZE set) the
ranks are used as they are; `python bench.py --gpus N` alone starts the N rank processes
itself (spawn, before anything touches a GPU).  The coarse quantizer is trained once on rank 0 and
broadcast; rank r generates the generator blocks b % N == r.  Default partition (--shard lists,
SURVEY.md 8(e)(i)): IVF lists shard WHOLE across the ranks (size-balanced, dist.list_owners); the
rows are exchanged to their list's owner (RCCL all_to_all, label order kept) and every rank holds a
replicated sample of every list.  A step (pyrope_amd.dist.ListShardedIvf) plans each rank's 10,000
home queries (coarse ranking + threshold), all_gathers the plans, scans on every rank only the
(query, list) pairs of its own lists, all_to_alls one record per query (exact local top-k + bound)
to the query's home, merges + certifies there, and re-runs the (rare) failures exactly -- 4 RCCL
collectives, the device work between them replayed from hipGraphs.  --shard rows: round 4's
rows-within-list shards (every rank searches every query; A/B only).  Per-GPU queries are fixed
as N grows ("weak").

Besides the QPS line the JSON carries:
  roofline      the dominant kernel (IVF list scan) timed with HIP events on its own stream:
                unique algorithmic bytes (every probed list once + queries) per launch against
                the HBM peak; "mfma" gives the as-executed MFMA rate
  cpu_baseline  the CPU restatement (oracle/, the reference's algorithm) on the host cores, on
                a bounded query sample of the same index (N = 1 only); its answers are also
                compared with the GPU's (ids equal, scores bit-identical)
  recall_at_10  vs the exact FLAT top-10 over the full data (per-rank FLAT shards + merge)
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

FP32_PEAK_TFLOPS = 157.3   # MI355X FP32 vector == FP32 matrix peak (MI355X_MICROARCH.md)
BF16_PEAK_TFLOPS = 2500.0  # dense bf16 MFMA peak (MI355X_MICROARCH.md, no sparsity)
HBM_PEAK_GBS = 8000.0      # HBM3E spec peak


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--n", type=int, default=10_000_000)
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--nlist", type=int, default=1024)
    ap.add_argument("--nprobe", type=int, default=32)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--nq", type=int, default=10_000, help="queries per GPU per step")
    ap.add_argument("--block-rows", type=int, default=65536, help="generator block (sharding unit)")
    ap.add_argument("--train-rows", type=int, default=10_000_000,
                    help="k-means runs on the first min(N, this) rows (all of I1)")
    ap.add_argument("--add-rows", type=int, default=2_000_000, help="rows per bulk add call")
    ap.add_argument("--recall-queries", type=int, default=1000)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline time (0 = skip)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = every CPU this process may use")
    ap.add_argument("--profile-steps", type=int, default=3)
    ap.add_argument("--shard", choices=["lists", "rows"], default="lists",
                    help="N > 1 partition: whole IVF lists per rank (default) or rows within lists (round 4, A/B)")
    ap.add_argument("--fcap", type=int, default=256, help="list-sharded: certificate failures a home re-runs per step")
    ap.add_argument("--graph", type=int, default=1,
                    help="N = 1: replay each step from a HIP graph of the whole search (1, default) or launch it "
                         "kernel by kernel (0); every replay runs every kernel of the search")
    return ap.parse_args(argv)


# ---------------------------------------------------------------------------------------------
# host CPU description for cpu_baseline ("report the lscpu model, sockets, cores")
# ---------------------------------------------------------------------------------------------
def cgroup_cpu_quota():
    """CPUs granted by a cgroup v2 (cpu.max) or v1 (cfs quota) limit, or None."""
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            return float(q) / float(p)
    except (OSError, ValueError):
        pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        p = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        if q > 0:
            return q / p
    except (OSError, ValueError):
        pass
    return None


def host_cpus():
    info = {"cpu_count": os.cpu_count()}
    try:
        info["affinity"] = len(os.sched_getaffinity(0))
    except AttributeError:
        info["affinity"] = os.cpu_count()
    quota = cgroup_cpu_quota()
    info["cgroup_quota_cpus"] = quota
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            k, _, v = line.partition(":")
            k, v = k.strip(), v.strip()
            if k in ("Model name", "Socket(s)", "Core(s) per socket", "Thread(s) per core", "CPU(s)"):
                info[{"Model name": "model", "Socket(s)": "sockets", "Core(s) per socket": "cores_per_socket",
                      "Thread(s) per core": "threads_per_core", "CPU(s)": "lscpu_cpus"}[k]] = v
    except (OSError, subprocess.SubprocessError):
        pass
    usable = info["affinity"] or 1
    if quota:
        usable = max(1, min(usable, int(quota)))
    info["usable"] = usable
    return info


# ---------------------------------------------------------------------------------------------
# rank processes
# ---------------------------------------------------------------------------------------------
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_entry(rank, world, port, argv):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    run(parse(argv))


def spawn_ranks(args, argv):
    """`--gpus N` without a launcher: N fresh rank processes (this process never touches a GPU).
    The library is built here first (hipcc needs no GPU), so the ranks find it current."""
    import torch.multiprocessing as mp
    from pyrope_amd.build import build
    build()
    log(f"--gpus {args.gpus} without a launcher: starting {args.gpus} rank processes")
    mp.start_processes(_rank_entry, args=(args.gpus, _free_port(), argv), nprocs=args.gpus, join=True,
                       start_method="spawn")


# ---------------------------------------------------------------------------------------------
# the benchmark proper (one rank)
# ---------------------------------------------------------------------------------------------
def run(args):
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    # PYR_BENCH_REHEARSE=1 (rehearsal only, never a reported line): every rank on cuda:0 over gloo, so the
    # N > 1 step runs end to end on a one-GPU box (RCCL refuses two ranks on one device)
    rehearse = world > 1 and os.environ.get("PYR_BENCH_REHEARSE") == "1"
    local = 0 if rehearse else int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)

    from pyrope_amd import (BruteForceVectorIndex, IvfFlatVectorIndex, VectorMetric, _lib, generate_synthetic,
                            generate_synthetic_blocked, kmeans_train)
    from pyrope_amd.build import build
    from pyrope_amd.dist import (Comm, DeviceShardEngine, ListShardedIvf, ShardedIvfStep, all_gather_rows,
                                 exchange_rows, gather_partials, gather_samples, merge_device, shard_blocks)
    from pyrope_amd.vector import SearchOptions
    build()
    L = _lib.load()

    D, N, k, B = args.dim, args.n, args.k, args.block_rows
    blocks = shard_blocks(N, world, rank, B)

    def shard_chunks():
        """(labels, rows) of this rank's blocks, <= add_rows rows per chunk (regenerated on demand)."""
        i = 0
        while i < len(blocks):
            j, rows = i, 0
            while j < len(blocks) and (rows == 0 or rows + blocks[j][1] - blocks[j][0] <= args.add_rows):
                rows += blocks[j][1] - blocks[j][0]
                j += 1
            labs = np.concatenate([np.arange(a, b, dtype=np.int64) for a, b in blocks[i:j]])
            x = np.concatenate([generate_synthetic_blocked(a, b - a, D, 42, B) for a, b in blocks[i:j]])
            yield labs, x
            i = j

    # 1) the coarse quantizer: KMeansUtils.Train (IvfFlatVectorIndex.Build, seed 42) over the first
    #    min(N, train_rows) rows, once, on rank 0; every shard builds with the same centroids
    T = min(N, args.train_rows)
    nl = max(1, min(args.nlist, T))
    ct = torch.empty((nl, D), dtype=torch.float32, device=dev)
    if rank == 0:
        t = time.time()
        train = generate_synthetic_blocked(0, T, D, 42, B)
        cents = kmeans_train(train, args.nlist, VectorMetric.L2, 10, 42, device=local)
        del train
        assert cents.shape == (nl, D)
        ct.copy_(torch.from_numpy(cents))
        log(f"k-means nlist={nl} over {T} rows in {time.time() - t:.1f}s")
    if world > 1:
        dist.broadcast(ct, 0)
    cents = ct.cpu().numpy()

    # 2) this rank's shard (IvfFlat Add into the buffer, then Build = assignment with the given quantizer)
    t = time.time()
    idx = IvfFlatVectorIndex(D, VectorMetric.L2, n_list=args.nlist, device=local)
    idx.set_centroids(cents)
    keep = world == 1 and args.cpu_seconds > 0  # the CPU baseline reads base rows
    kept = []
    nrows = 0
    lists_sharded = world > 1 and args.shard == "lists"
    comm = Comm(world)
    if lists_sharded:
        # whole lists: every row to its list's owner (label order kept), then the replicated list samples
        added = [0]

        def add(labs, x):
            idx.add_labels(labs, x, track_ids=False)
            added[0] += len(labs)
        glen, owner, samples = exchange_rows(comm, rank, world, shard_chunks, cents, VectorMetric.L2, device=local,
                                             add=add)
        nrows = added[0]
        idx.build()
        srows, scounts = gather_samples(comm, rank, world, glen, owner, samples, D)
        idx.set_list_samples(srows, scounts, glen)
        del srows, samples
        log(f"rank {rank}: {int((owner == rank).sum())} whole lists, {nrows} rows (rank rows max/min "
            f"{np.bincount(owner, weights=glen, minlength=world).max():.0f}/"
            f"{np.bincount(owner, weights=glen, minlength=world).min():.0f})")
    else:
        for labs, x in shard_chunks():
            idx.add_labels(labs, x, track_ids=False)
            nrows += len(labs)
            if keep:
                kept.append(x)
            if nrows % (5 * args.add_rows) < len(labs):  # progress for long (M8-size) loads
                log(f"rank {rank}: {nrows} rows added ({time.time() - t:.0f}s)")
        idx.build()
    data = np.concatenate(kept) if keep else None  # world == 1: rows in base-row (= label) order
    del kept
    log(f"rank {rank}: shard of {nrows} rows ({len(blocks)} blocks) generated + indexed in {time.time() - t:.1f}s")

    Q = args.nq * world
    qh = generate_synthetic(Q, D, 1337)
    q = torch.from_numpy(qh).to(dev)
    opts = SearchOptions(nprobe=args.nprobe)
    width = max(0, min(args.nprobe, nl))
    s_loc = torch.empty((Q, k), dtype=torch.float32, device=dev)
    l_loc = torch.empty((Q, k), dtype=torch.int64, device=dev)
    pr_loc = torch.empty((args.nq, width), dtype=torch.int32, device=dev)
    result = [s_loc, l_loc]

    def probe(qs):  # this rank's slice of the batch (pyr_index_probe_device)
        w = idx.probe_device(qs.data_ptr(), qs.shape[0], pr_loc.data_ptr(), torch.cuda.current_stream().cuda_stream,
                             opts)
        assert w == width
        return pr_loc

    def search(qs, probes):  # every query against this rank's shard, the gathered probe lists
        idx.search_device(qs.data_ptr(), qs.shape[0], k, s_loc.data_ptr(), l_loc.data_ptr(), 0,
                          torch.cuda.current_stream().cuda_stream, opts, d_probes=probes.data_ptr(), nprobe=width)
        return s_loc, l_loc

    def merge(sp, lp, kk):  # RCCL all_gather'ed partial top-k [world, Q, k] -> on-device merge
        return merge_device(sp, lp, kk, torch.cuda.current_stream().cuda_stream, part_major=True)

    # the N > 1 step's buffers: allocated once, reused by every step
    sharded = None
    if world > 1 and lists_sharded:
        sharded = ListShardedIvf(DeviceShardEngine(idx, k, opts), comm, args.nq, k, width, rank, world, device=dev,
                                 fcap=args.fcap)
    elif world > 1:
        sharded = ShardedIvfStep(args.nq, width, k, rank, world, device=dev)

    def step():
        if world == 1:
            idx.search_device(q.data_ptr(), Q, k, s_loc.data_ptr(), l_loc.data_ptr(), 0,
                              torch.cuda.current_stream().cuda_stream, opts)
            return
        if lists_sharded:
            result[:] = sharded(q)
            return
        result[:] = sharded(q, probe, search, merge)

    def barrier():
        if world > 1:
            dist.barrier()

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    timed_step = step
    graph = None
    if world == 1 and args.graph:
        # the whole search (coarse ranking .. exact re-run) captured once on a side stream: the workspace
        # is sized by the warm-up, pyr_index_search_device only enqueues (no host sync, no allocation),
        # and a replay launches every kernel of the step with its launch gaps removed
        gst = torch.cuda.Stream()
        gst.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(gst):
            step()  # the capture stream's own workspace
        gst.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=gst):
            step()
        torch.cuda.synchronize()
        # untimed replays: at least W, and for at least 50 ms -- the capture leaves the GPU idle for ~15 ms and
        # its clocks then take ~10 steps to return (the first timed replays of a 20-step region ran 1.5-1.7 ms
        # instead of 1.25 ms, profiles/r5_start/kt20_steps.txt)
        t_w = time.perf_counter()
        n_w = 0
        while n_w < max(1, args.warmup) or time.perf_counter() - t_w < 0.05:
            graph.replay()
            n_w += 1
            if n_w % 8 == 0:
                torch.cuda.synchronize()
        torch.cuda.synchronize()
        timed_step = graph.replay
    elif lists_sharded and args.graph:
        # the device work between the collectives replayed from hipGraphs (ListShardedIvf.capture); every
        # rank runs the same number of untimed steps (they synchronize in the collectives)
        sharded.capture(q)
        graph = sharded.graphs
        n_w = max(10, args.warmup)
        for _ in range(n_w):
            step()
        torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        timed_step()
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    # the timed replays' answer (the last replay's results) against a plain kernel-by-kernel search of the same
    # batch: bit-identical, so the graph replays computed the search (DESIGN.md §4 "hipGraph replays")
    graph_check = None
    if graph is not None:
        o_s, o_l = (s_loc, l_loc) if world == 1 else (result[0], result[1])
        g_s, g_l = o_s.clone(), o_l.clone()
        o_s.fill_(0.0)
        o_l.fill_(-7)
        if world > 1:
            saved, sharded.graphs = sharded.graphs, {}
            step()
            sharded.graphs = saved
        else:
            step()
        torch.cuda.synchronize()
        graph_check = {"replays": args.steps + n_w, "untimed_replays": n_w,
                       "last_replay_equals_direct_search": bool(torch.equal(g_l, o_l)) and
                       bool(torch.equal(g_s.view(torch.int32), o_s.view(torch.int32)))}
        log(f"graph replay vs direct search: {graph_check}")
    if world > 1:
        e = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
    qps = Q * args.steps / elapsed
    log(f"rank {rank}: {args.steps} steps in {elapsed * 1e3:.1f} ms -> {qps:,.0f} QPS")

    # ---- per-phase kernel times (HIP events on the search stream), outside the timed region ----
    phases = {}
    coll = {}
    L.pyr_profile_reset()
    L.pyr_profile_enable(1)
    saved_graphs = None
    if lists_sharded and getattr(sharded, "graphs", None):
        saved_graphs, sharded.graphs = sharded.graphs, {}  # the per-phase profile needs the plain launches
    if sharded is not None:
        sharded.timing = True
    for _ in range(args.profile_steps):
        step()
        if sharded is not None:
            for kk, v in sharded.collective_ms.items():
                coll[kk] = coll.get(kk, 0.0) + v / args.profile_steps
    torch.cuda.synchronize()
    L.pyr_profile_enable(0)
    if sharded is not None:
        sharded.timing = False
    if saved_graphs is not None:
        sharded.graphs = saved_graphs
    # rows of every rank's shard (weak scaling: each rank holds N / world of them)
    rank_rows = [nrows]
    if world > 1:
        rank_rows = all_gather_rows(torch.tensor([nrows], dtype=torch.int64, device=dev), world).cpu().tolist()
    import ctypes as C
    names = {0: "coarse", 1: "work_lists", 9: "sample", 2: "list_scan", 3: "buffer_scan", 4: "merge", 7: "refine",
             8: "exact_rerun"}
    fallback_queries = 0
    for ph, name in names.items():
        ms, calls, work = C.c_double(), C.c_int64(), C.c_int64()
        L.pyr_profile_get(ph, C.byref(ms), C.byref(calls), C.byref(work))
        if calls.value:
            phases[name] = {"ms": ms.value / calls.value, "pairs": work.value // calls.value}
        if ph == 8:
            fallback_queries = work.value
    scan = phases.get("list_scan", {"ms": float("nan"), "pairs": 0})
    # (the library honours PYR_FILTER only with PYR_DEV_KNOBS=1, kernels.h knob())
    filt = not (os.environ.get("PYR_DEV_KNOBS") == "1" and os.environ.get("PYR_FILTER", "1") == "0")
    # MFMA filter (default): the (query, row) GEMM, 2*D flops per pair; exact VALU scan
    # (PYR_FILTER=0): sub, mul, add per element, 3*D
    flops = scan["pairs"] * (2 if filt else 3) * D
    achieved = flops / (scan["ms"] * 1e-3) / 1e12
    # the list-scan kernel (engine.cpp search_stream): the stream-and-emit scan (scan.hip), one fp16 MFMA
    # per 16-dim k-step; PYR_FILTER=0: the exact VALU scan (kernels.hip scan_fast)
    prec = 3 if filt else -1
    if filt:
        mfma_mult, mfma_peak = 1, BF16_PEAK_TFLOPS
        kernel_tag = "scan32"
        kernel_name = (f"scan_kernel<{D},L2> (scan.hip: IVF list scan, stream-and-emit over fp16 residual tiles: "
                       f"persistent 16-wave blocks, tiles from HBM into registers as the A operand of "
                       f"v_mfma_f32_32x32x16_f16, queries from LDS, one MFMA per 16-dim k-step)")
    else:
        kernel_tag = "scan_fast"
        mfma_mult, mfma_peak = 1, FP32_PEAK_TFLOPS
        kernel_name = "scan_fast<128,1,L2,IVF> (IVF list scan, exact VALU)"
    # unique algorithmic bytes of one list-scan launch on this rank: every list probed by any query
    # of the batch read once (its live rows of this shard x D x 4 B) plus the batch's queries -- the
    # HBM floor of a batched, list-major scan (SURVEY.md 8(d) "unique-bytes roofline")
    pr_full = torch.empty((Q, width), dtype=torch.int32, device=dev)
    idx.probe_device(q.data_ptr(), Q, pr_full.data_ptr(), 0, opts)
    torch.cuda.synchronize()
    off_l, lab_l, live_l = idx.ivf_layout()
    cs_live = np.concatenate([[0], np.cumsum(live_l.astype(np.int64))])
    rows_per_list = cs_live[off_l[1:]] - cs_live[off_l[:-1]]
    probed = np.unique(pr_full.cpu().numpy())
    probed = probed[probed >= 0]
    unique_bytes = float(rows_per_list[probed].sum()) * D * 4 + Q * D * 4
    # what the fp16 tile kernel streams for the same rows: D x 2 B + a 4-B row term, padded lists
    padded = np.diff(off_l).astype(np.int64)
    stored_bytes = float(padded[probed].sum()) * (D * 2 + 4) + Q * D * 4 if prec in (2, 3) else unique_bytes
    hbm_achieved = unique_bytes / (scan["ms"] * 1e-3) / 1e9
    del pr_full

    # ---- recall@10 vs the exact FLAT top-10 over all N rows: per-rank FLAT shard + merge ----
    recall = None
    truth_check = None
    s_fin = result[0].cpu().numpy()
    l_fin = result[1].cpu().numpy()
    if args.recall_queries > 0:
        t = time.time()
        R = min(args.recall_queries, Q, len(l_fin))  # list-sharded: rank 0 answers its home queries
        flat = BruteForceVectorIndex(D, VectorMetric.L2, device=local)
        for labs, x in shard_chunks():
            flat.add_labels(labs, x, track_ids=False)
        fs, fl, _ = flat.search_batch(qh[:R], k)
        flat.close()
        gs, gl = torch.from_numpy(fs).to(dev), torch.from_numpy(fl).to(dev)
        if world > 1:
            sp, lp = gather_partials(gs, gl, world)
            gs, gl = merge_device(sp, lp, k, torch.cuda.current_stream().cuda_stream)
        gt = gl.cpu().numpy()
        if rank == 0 or not lists_sharded:  # list-sharded: rank 0 holds the answers of queries [0, nq)
            hits = sum(len(set(gt[i].tolist()) & set(l_fin[i].tolist())) for i in range(R))
            recall = hits / (R * k)
            log(f"recall@10 over {R} queries: {recall:.4f} ({time.time() - t:.1f}s)")
        # the ground truth itself against the CPU restatement of BruteForceVectorIndex.Search (checker only)
        if rank == 0 and world == 1 and args.cpu_seconds > 0 and data is not None:
            import oracle  # checker only
            G = min(64, R)
            t = time.time()
            os_, ok_, _ = oracle.bf_search_batch(qh[:G], k, data, nthreads=args.cpu_threads or host_cpus()["usable"])
            truth_check = {"queries": G, "ids_equal": bool(np.array_equal(ok_, fl[:G])),
                           "scores_bit_identical": bool(np.array_equal(os_.view(np.uint32), fs[:G].view(np.uint32))),
                           "note": "GPU FLAT ground truth of the first queries vs oracle/oracle.c BruteForce search "
                                   "over all N rows"}
            log(f"recall ground truth vs CPU oracle: {G} queries, ids {truth_check['ids_equal']}, bits "
                f"{truth_check['scores_bit_identical']} ({time.time() - t:.1f}s)")

    # ---- CPU baseline: the oracle (CPU restatement of the reference engine) on the same index ----
    cpu = None
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        import oracle  # checker / CPU baseline only
        host = host_cpus()
        threads = args.cpu_threads or host["usable"]
        lab_rows = np.where(lab_l >= 0, lab_l, 0)  # list-major position -> base row (labels are row ids)
        # list-major copy of the rows when it fits (contiguous list scans: the faster CPU baseline), else
        # the base rows read through the layout's row index
        lrows = data[lab_rows] if data.nbytes <= (16 << 30) else None

        def cpu_run(S):
            if lrows is not None:
                return oracle.ivf_search_batch(qh[:S], k, cents, lrows, off_l, live_l, nprobe=args.nprobe,
                                               nthreads=threads)
            return oracle.ivf_search_batch_idx(qh[:S], k, cents, data, lab_rows, off_l, live_l, nprobe=args.nprobe,
                                               nthreads=threads)
        S = min(Q, 4 * threads)
        t = time.perf_counter()
        cpu_run(S)
        probe_t = time.perf_counter() - t
        S = int(min(Q, max(S, S * args.cpu_seconds / max(probe_t, 1e-3))))
        t = time.perf_counter()
        cs, ck, cc = cpu_run(S)
        ct_ = time.perf_counter() - t
        ids_equal = bool(np.array_equal(np.where(ck >= 0, lab_l[np.maximum(ck, 0)], -1), l_fin[:S]))
        bits_equal = bool(np.array_equal(cs.view(np.uint32), s_fin[:S].view(np.uint32)))
        cpu = {"value": S / ct_, "unit": "queries/s", "cores": threads, "kind": "port",
               # per thread: the figure that compares box to box (the whole-host rate moves with the quota and
               # the other tenants of the box's cores)
               "per_thread_qps": S / ct_ / max(threads, 1),
               "sample": f"{S} of the {Q} batch queries, same index (oracle/oracle.c IVF search, one query per "
                         f"thread, {threads} threads = every CPU this process may use, {ct_:.1f}s)",
               "host": host,
               "parity": {"queries": S, "ids_equal": ids_equal, "scores_bit_identical": bits_equal}}
        log(f"cpu baseline: {S / ct_:,.1f} QPS on {threads} threads ({host.get('model')}); "
            f"parity ids={ids_equal} bits={bits_equal}")

    # roofline traffic: HBM bytes per list-scan launch from the committed FETCH_SIZE counter pass
    # (traffic.json; counters need their own rocprofv3 run), used only for the configuration and the
    # list-scan arithmetic it was measured on
    traffic, traffic_src = None, None
    tpath = os.path.join(os.path.dirname(os.path.abspath(__file__)), "traffic.json")
    if os.path.exists(tpath) and world == 1:
        tj = json.load(open(tpath))
        tc = tj.get("config", {})
        same_kernel = tj.get("kernel_tag") == kernel_tag
        if same_kernel and (tc.get("n"), tc.get("dim"), tc.get("nlist"), tc.get("nprobe"), tc.get("k"),
                            tc.get("nq")) == (N, D, args.nlist, args.nprobe, k, args.nq):
            traffic, traffic_src = tj["hbm_read_bytes_per_launch"], tj["source"]

    # list-sharded: the (query, list) pairs each rank scanned in the last step (every query of the batch,
    # its probe lists from the all_gather'ed plan, counted by list owner) -- the per-rank work balance
    pair_balance = None
    if lists_sharded:
        own = torch.from_numpy(owner.astype(np.int64)).to(dev)
        pl = sharded.plan_all[:, :width].long()
        per = torch.bincount(own[pl[pl >= 0]], minlength=world).cpu().tolist()
        pair_balance = {"pairs_per_rank": per, "max_over_mean": max(per) / (sum(per) / world),
                        "rows_per_rank": rank_rows,
                        "note": "(query, probed list) pairs of the whole batch by the rank owning the list"}
    # list-sharded: the bytes each collective moves per rank per step (what a rank sends; an all_gather's
    # output is world x its input), and the certificate failures of the home ranks (every one is re-run:
    # rounds of fcap per home, ListShardedIvf)
    shard_messages = shard_cert = None
    if lists_sharded:
        rb = 16 * (k + 1)
        S = sharded.plan_home.shape[1]
        shard_messages = {"plan_allgather_in": args.nq * S * 4, "record_alltoall_send": Q * rb,
                          "fail_allgather_in": (1 + sharded.fcap) * 4, "rerun_alltoall_send": world * sharded.fcap * rb,
                          "unit": "bytes per rank per step"}
        shard_cert = {"fcap": sharded.fcap, "max_failures_per_home": sharded.max_fail,
                      "extra_rounds_last_step": sharded.stats["extra_rounds"],
                      "note": "certificate failures at one home rank over every step run (all ranks see every "
                              "home's count); failures past fcap are re-run in further rounds"}
    if rank == 0:
        bytes_per_query = args.nprobe / args.nlist * N * D * 4 + args.nlist * D * 4
        out = {
            "metric": "QPS + recall@10, IVF-Flat d=128 N=10M nprobe=32 at 1/2/4/8 MI355X",
            "value": qps,
            "unit": "queries/s",
            "n_gpus": world,
            "ranks_seen": dist.get_world_size() if world > 1 else 1,
            "backend": (dist.get_backend() + (" (RCCL)" if dist.get_backend() == "nccl" else " (rehearsal: one GPU)"))
                       if world > 1 else None,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",  # results and the certified refine are fp32; the filter streams fp16 tiles
            "data": "synthetic: Pyrope.Benchmarks generator (.NET Random), base rows in 65,536-row blocks seeded "
                    "42 + block, queries seed 1337, uniform [0,1)",
            "config": {"workload": f"IVF_FLAT d={D} N={N} nlist={args.nlist} nprobe={args.nprobe} k={k}",
                       "n": N, "dim": D, "nlist": args.nlist, "nprobe": args.nprobe, "k": k,
                       "queries_per_step": Q, "queries_per_gpu": args.nq, "train_rows": T,
                       "shard": ("whole IVF lists per rank (size-balanced), rows exchanged to their list's owner, "
                                 "replicated list samples; shared quantizer (trained on rank 0, broadcast)"
                                 if lists_sharded else
                                 "rows-within-list: generator blocks b % n_gpus == rank, shared quantizer "
                                 "(trained on rank 0, broadcast)") if world > 1 else "none",
                       "merge": ("RCCL all_gather of plans, all_to_all of per-query records to their home rank, "
                                 "on-device merge + certificate, exact re-run of failures (all_gather + all_to_all)"
                                 if lists_sharded else
                                 "RCCL all_gather of probe lists and of partial top-k + on-device merge")
                                if world > 1 else "none"},
            "recall_at_10": recall,
            "recall_truth_check": truth_check,
            "roofline": {"bound": "hbm", "achieved": hbm_achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": hbm_achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "traffic_source": traffic_src,
                         # the bytes the kernel physically moved (FETCH_SIZE pass) at this launch's time
                         "frac_physical": (traffic / (scan["ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS) if traffic else None,
                         "unique_bytes_per_launch": unique_bytes, "lists_probed": int(len(probed)),
                         "kernel": kernel_name,
                         "stored_bytes_per_launch": stored_bytes,
                         "stored_GBps": stored_bytes / (scan["ms"] * 1e-3) / 1e9,
                         "stored_frac": stored_bytes / (scan["ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS,
                         "note": ("algorithmic bytes = every probed list read once per launch (live rows x D x "
                                  "4 B, the reference's fp32 rows) + queries, over the HIP-event time of the launch "
                                  "(rank 0); stored_bytes = what the fp16 tile kernel actually streams for them "
                                  "(D x 2 + 4 B per padded row), stored_frac = their rate vs the peak; traffic (FETCH_SIZE x 2, its "
                                  "own rocprofv3 pass, per launch; traffic.json) and frac_physical = traffic over the same "
                                  "launch time vs the peak")},
            "mfma": {"achieved": achieved * mfma_mult, "peak": mfma_peak, "unit": "TFLOP/s",
                     "frac": achieved * mfma_mult / mfma_peak,
                     "note": (f"as-executed MFMA flops: probed (query,row) pairs x 2*D x {mfma_mult} (MFMAs per "
                              f"k-step) vs the dense fp16/bf16 peak" if prec in (1, 2, 3) else
                              "probed pairs x 2*D (fp32 MFMA) or x 3*D (exact VALU) vs the FP32 peak")},
            "exact_reruns": {"queries": fallback_queries, "in_profiled_steps": args.profile_steps,
                             "note": "queries whose MFMA-filter certificate failed and were re-scanned exactly"},
            "per_query_bytes": {"bytes_per_query": bytes_per_query,
                                "note": "SURVEY.md 8(d): nprobe/nlist x N x D x 4 + nlist x D x 4 per query (no "
                                        "batching reuse); not a roofline"},
            "launch": "hipGraph replay of the whole search per step" if graph is not None else "kernel launches",
            "graph_check": graph_check,
            "phases_ms": {k_: round(v["ms"], 4) for k_, v in phases.items()},
            "collective_ms": {k_: round(v, 4) for k_, v in coll.items()} if world > 1 else None,
            "rank_rows": rank_rows,
            "pair_balance": pair_balance,
            "shard_messages": shard_messages,
            "shard_certificate": shard_cert,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    idx.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def main():
    argv = sys.argv[1:]
    args = parse(argv)
    if args.gpus > 1 and "RANK" not in os.environ and int(os.environ.get("WORLD_SIZE", "1")) <= 1:
        spawn_ranks(args, argv)
        return
    run(args)


if __name__ == "__main__":
    main()
