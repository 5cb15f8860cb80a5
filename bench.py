#!/usr/bin/env python3
"""bench.py -- QPS + recall@10 of the IVF_FLAT scan on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[2]): IVF_FLAT d=128, N=10M base vectors, nlist=1024,
nprobe=32, top-10, synthetic uniform [0,1) vectors from the reference benchmark's
generator (Pyrope.Benchmarks/Program.cs:251-263: base seed 42, query seed 1337).

A step = one batched search of the query batch (10,000 queries per GPU), queries
and results resident in HBM.  With --gpus N (one process per GPU, RCCL), the
index is sharded rows-within-list (every rank holds row i iff i % N == rank, all
ranks share one coarse quantizer), every rank scans its shard for the global
batch (10,000 x N queries), and partial top-k lists are merged after an RCCL
all_gather: per-GPU work is fixed as N grows ("weak").

Besides the QPS line the JSON carries:
  roofline      the dominant kernel (IVF list scan) timed with HIP events on its own
                stream: unique algorithmic bytes (every probed list once + queries) per
                launch against the HBM peak; "mfma" gives the as-executed MFMA rate
  cpu_baseline  the CPU restatement (oracle/, the reference's algorithm) on the host
                cores, on a bounded query sample of the same index; its answers are also
                compared with the GPU's (ids equal, scores bit-identical)
  recall_at_10  vs exact FLAT top-10 over the full data (GPU FLAT index)
"""
from __future__ import annotations

import argparse
import json
import os
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


def main():
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
    ap.add_argument("--recall-queries", type=int, default=1000)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline time (0 = skip)")
    ap.add_argument("--profile-steps", type=int, default=3)
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    from pyrope_amd import IvfFlatVectorIndex, VectorMetric, generate_synthetic, kmeans_train, _lib
    from pyrope_amd.build import build
    build()
    L = _lib.load()

    D, N, k = args.dim, args.n, args.k
    t = time.time()
    data = generate_synthetic(N, D, 42)  # every rank regenerates the same base set
    log(f"rank {rank}: generated {N}x{D} in {time.time() - t:.1f}s")
    t = time.time()
    cents = kmeans_train(data, args.nlist, VectorMetric.L2, 10, 42, device=local)  # IvfFlat.Build: seed 42
    log(f"rank {rank}: k-means nlist={len(cents)} in {time.time() - t:.1f}s")
    t = time.time()
    idx = IvfFlatVectorIndex(D, VectorMetric.L2, n_list=args.nlist, device=local)
    idx.set_centroids(cents)
    from pyrope_amd.dist import shard_labels
    shard = shard_labels(N, world, rank)
    idx.add_labels(shard, data[rank::world])
    idx.build()
    log(f"rank {rank}: shard of {len(shard)} rows indexed in {time.time() - t:.1f}s")

    Q = args.nq * world
    qh = generate_synthetic(Q, D, 1337)
    q = torch.from_numpy(qh).to(dev)
    s_loc = torch.empty((Q, k), dtype=torch.float32, device=dev)
    l_loc = torch.empty((Q, k), dtype=torch.int64, device=dev)
    from pyrope_amd.dist import gather_partials, merge_device
    from pyrope_amd.vector import SearchOptions
    opts = SearchOptions(nprobe=args.nprobe)
    result = [s_loc, l_loc]

    # N > 1: the coarse ranking is split too -- rank r ranks the quantizer for its own nq-query
    # slice of the batch and one all_gather assembles every query's probe lists -- so per-GPU
    # work stays fixed as N grows (every rank would otherwise rank the whole N x nq batch)
    pr_loc = torch.empty((args.nq, args.nprobe), dtype=torch.int32, device=dev)
    pr_all = torch.empty((Q, args.nprobe), dtype=torch.int32, device=dev)

    def step():
        stream = torch.cuda.current_stream().cuda_stream
        if world == 1:
            idx.search_device(q.data_ptr(), Q, k, s_loc.data_ptr(), l_loc.data_ptr(), 0, stream, opts)
            return
        q_mine = q[rank * args.nq:(rank + 1) * args.nq]
        width = idx.probe_device(q_mine.data_ptr(), args.nq, pr_loc.data_ptr(), stream, opts)
        dist.all_gather_into_tensor(pr_all, pr_loc)
        idx.search_device(q.data_ptr(), Q, k, s_loc.data_ptr(), l_loc.data_ptr(), 0, stream, opts,
                          d_probes=pr_all.data_ptr(), nprobe=width)
        # RCCL all_gather over xGMI of per-GPU partial top-k, then on-device merge
        sp, lp = gather_partials(s_loc, l_loc, world)
        result[:] = merge_device(sp, lp, k, stream)

    def barrier():
        if world > 1:
            dist.barrier()

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        e = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
    qps = Q * args.steps / elapsed
    log(f"rank {rank}: {args.steps} steps in {elapsed * 1e3:.1f} ms -> {qps:,.0f} QPS")

    # ---- per-phase kernel times (HIP events on the search stream), outside the timed region ----
    phases = {}
    L.pyr_profile_reset()
    L.pyr_profile_enable(1)
    for _ in range(args.profile_steps):
        step()
    torch.cuda.synchronize()
    L.pyr_profile_enable(0)
    import ctypes as C
    names = {0: "coarse", 1: "work_lists", 2: "list_scan", 3: "buffer_scan", 4: "merge", 7: "refine",
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
    filt = os.environ.get("PYR_FILTER", "1") != "0"
    # MFMA filter (default): the (query, row) GEMM, 2*D flops per pair; exact VALU scan
    # (PYR_FILTER=0): sub, mul, add per element, 3*D
    flops = scan["pairs"] * (2 if filt else 3) * D
    achieved = flops / (scan["ms"] * 1e-3) / 1e12
    bf16x3 = filt and os.environ.get("PYR_FILTER_PREC", "1") != "0"
    # unique algorithmic bytes of one list-scan launch: every list probed by any query of the
    # batch read once (its live rows x D x 4 B) plus the batch's queries -- the HBM floor of a
    # batched, list-major scan (SURVEY.md 8(d) "unique-bytes roofline")
    pr_full = torch.empty((Q, args.nprobe), dtype=torch.int32, device=dev)
    width = idx.probe_device(q.data_ptr(), Q, pr_full.data_ptr(), 0, opts)
    torch.cuda.synchronize()
    off_l, lab_l, live_l = idx.ivf_layout()
    cs_live = np.concatenate([[0], np.cumsum(live_l.astype(np.int64))])
    rows_per_list = cs_live[off_l[1:]] - cs_live[off_l[:-1]]
    probed = np.unique(pr_full[:, :width].cpu().numpy())
    probed = probed[probed >= 0]
    unique_bytes = float(rows_per_list[probed].sum()) * D * 4 + Q * D * 4
    hbm_achieved = unique_bytes / (scan["ms"] * 1e-3) / 1e9

    # ---- recall@10 vs exact FLAT top-10 (rank 0) ----
    recall = None
    s_fin = result[0].cpu().numpy()
    l_fin = result[1].cpu().numpy()
    if rank == 0 and args.recall_queries > 0:
        from pyrope_amd import BruteForceVectorIndex
        R = min(args.recall_queries, Q)
        flat = BruteForceVectorIndex(D, VectorMetric.L2, device=local)
        flat.add_labels(np.arange(N, dtype=np.int64), data)
        _, gt, _ = flat.search_batch(qh[:R], k)
        flat.close()
        hits = sum(len(set(gt[i].tolist()) & set(l_fin[i].tolist())) for i in range(R))
        recall = hits / (R * k)
        log(f"recall@10 over {R} queries: {recall:.4f}")

    # ---- CPU baseline: the oracle (CPU restatement of the reference engine) on the same index ----
    cpu = None
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        import oracle  # checker / CPU baseline only
        off, labels, live = idx.ivf_layout()
        rows = data[labels]
        cts = idx.centroids_array()
        threads = max(1, min(16, os.cpu_count() or 1))
        S = min(Q, 4 * threads)
        t = time.perf_counter()
        oracle.ivf_search_batch(qh[:S], k, cts, rows, off, live, nprobe=args.nprobe, nthreads=threads)
        probe = time.perf_counter() - t
        S = int(min(Q, max(S, S * args.cpu_seconds / max(probe, 1e-3))))
        t = time.perf_counter()
        cs, ck, cc = oracle.ivf_search_batch(qh[:S], k, cts, rows, off, live, nprobe=args.nprobe, nthreads=threads)
        ct = time.perf_counter() - t
        ids_equal = bool(np.array_equal(labels[ck], l_fin[:S]))
        bits_equal = bool(np.array_equal(cs.view(np.uint32), s_fin[:S].view(np.uint32)))
        cpu = {"value": S / ct, "unit": "queries/s", "cores": threads, "kind": "port",
               "sample": f"{S} of the {Q} batch queries, same index (oracle/oracle.c IVF search, "
                         f"one query per thread, {threads} threads, {ct:.1f}s)",
               "parity": {"queries": S, "ids_equal": ids_equal, "scores_bit_identical": bits_equal}}
        log(f"cpu baseline: {S / ct:,.1f} QPS on {threads} threads; parity ids={ids_equal} bits={bits_equal}")
        del rows

    if rank == 0:
        bytes_per_query = args.nprobe / args.nlist * N * D * 4 + args.nlist * D * 4
        out = {
            "metric": "QPS + recall@10, IVF-Flat d=128 N=10M nprobe=32 at 1/2/4/8 MI355X",
            "value": qps,
            "unit": "queries/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic: Pyrope.Benchmarks generator (.NET Random, base seed 42, query seed 1337), "
                    "uniform [0,1)",
            "config": {"workload": f"IVF_FLAT d={D} N={N} nlist={args.nlist} nprobe={args.nprobe} k={k}",
                       "n": N, "dim": D, "nlist": args.nlist, "nprobe": args.nprobe, "k": k,
                       "queries_per_step": Q, "queries_per_gpu": args.nq,
                       "shard": "rows-within-list (row i on rank i % n_gpus), shared quantizer",
                       "merge": "RCCL all_gather of partial top-k + on-device merge" if world > 1 else "none"},
            "recall_at_10": recall,
            "roofline": {"bound": "hbm", "achieved": hbm_achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": hbm_achieved / HBM_PEAK_GBS, "traffic": None,
                         "unique_bytes_per_launch": unique_bytes, "lists_probed": int(len(probed)),
                         "kernel": ("mfma_filter<128,L2,IVF> (IVF list scan, bf16x3 MFMA candidate filter)"
                                    if bf16x3 else
                                    "mfma_filter<128,L2,IVF> (IVF list scan, fp32 MFMA candidate filter)" if filt
                                    else "scan_fast<128,1,L2,IVF> (IVF list scan, exact VALU)"),
                         "note": ("algorithmic bytes = every probed list read once per launch (live rows x D x "
                                  "4 B) + queries, over the HIP-event time of the launch; traffic (FETCH_SIZE, "
                                  "measured in its own rocprofv3 pass) is in profiles/*/summary.md")},
            "mfma": {"achieved": achieved * (3 if bf16x3 else 1),
                     "peak": BF16_PEAK_TFLOPS if bf16x3 else FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": achieved * (3 if bf16x3 else 1) / (BF16_PEAK_TFLOPS if bf16x3 else FP32_PEAK_TFLOPS),
                     "note": ("as-executed bf16 MFMA flops: probed (query,row) pairs x 2*D x 3 (hi.hi, hi.lo, "
                              "lo.hi) vs the dense bf16 peak" if bf16x3 else
                              "probed pairs x 2*D (fp32 MFMA) or x 3*D (exact VALU) vs the FP32 peak")},
            "exact_reruns": {"queries": fallback_queries, "in_profiled_steps": args.profile_steps,
                             "note": "queries whose MFMA-filter certificate failed and were re-scanned exactly"},
            "hbm_equivalent": {"bytes_per_query": bytes_per_query,
                               "GBps": qps * bytes_per_query / 1e9 / world,
                               "frac_of_8TBps_per_gpu": qps * bytes_per_query / 1e9 / world / HBM_PEAK_GBS},
            "phases_ms": {k_: round(v["ms"], 4) for k_, v in phases.items()},
            "cpu_baseline": cpu,
        }
        print(json.dumps(out))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
