#!/usr/bin/env python3
"""Serving sweep of the request coalescer (pyr_index_set_coalescing) on the I1 index.

Client threads call IVectorIndex.Search-style host searches (pyr_index_search through the
Python shim, one call = `nq` queries) in a closed loop for a few seconds; reported per setting:
QPS (queries/s) and per-call latency p50 / p99.  With coalescing off every call is its own
device search; with it on, concurrent calls are merged into device batches of up to
--max-batch queries (max wait --wait-us).  Output: one JSON object (stdout).

    python scripts/bench_coalesce.py --n 10000000 > profiles/r2_coalesce/sweep.json
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=10_000_000)
    ap.add_argument("--nlist", type=int, default=1024)
    ap.add_argument("--nprobe", type=int, default=32)
    ap.add_argument("--seconds", type=float, default=3.0)
    ap.add_argument("--max-batch", type=int, default=4096)
    ap.add_argument("--wait-us", type=int, default=2000)
    args = ap.parse_args()
    import torch  # noqa: F401  (HIP runtime up first, like bench.py)
    torch.cuda.init()
    from pyrope_amd import IvfFlatVectorIndex, VectorMetric, generate_synthetic, generate_synthetic_blocked
    from pyrope_amd import kmeans_train
    from pyrope_amd.vector import SearchOptions
    D, k = 128, 10
    x = generate_synthetic_blocked(0, args.n, D, 42)
    cents = kmeans_train(x[:min(args.n, 10_000_000)], args.nlist, VectorMetric.L2, 10, 42)
    idx = IvfFlatVectorIndex(D, VectorMetric.L2, n_list=args.nlist)
    idx.set_centroids(cents)
    idx.add_labels(np.arange(args.n, dtype=np.int64), x, track_ids=False)
    idx.build()
    del x
    q = generate_synthetic(20_000, D, 1337)
    opts = SearchOptions(nprobe=args.nprobe)
    print(f"index ready: N={args.n}", file=sys.stderr, flush=True)

    def run(nq, threads, coalesce):
        idx.set_coalescing(args.max_batch, args.wait_us if coalesce else 0)
        lat = [[] for _ in range(threads)]
        stop = time.perf_counter() + args.seconds
        done = [0] * threads

        def worker(t):
            rng = np.random.default_rng(t)
            while time.perf_counter() < stop:
                a = int(rng.integers(0, len(q) - nq + 1))
                t0 = time.perf_counter()
                idx.search_batch(q[a:a + nq], k, opts)
                lat[t].append(time.perf_counter() - t0)
                done[t] += nq

        th = [threading.Thread(target=worker, args=(t,)) for t in range(threads)]
        t0 = time.perf_counter()
        for t in th:
            t.start()
        for t in th:
            t.join()
        wall = time.perf_counter() - t0
        all_lat = np.array([v for l in lat for v in l]) * 1e3
        return {"nq_per_call": nq, "threads": threads, "coalescing": coalesce, "qps": sum(done) / wall,
                "calls": int(all_lat.size), "p50_ms": float(np.percentile(all_lat, 50)),
                "p99_ms": float(np.percentile(all_lat, 99))}

    out = []
    for nq, threads in [(1, 64), (16, 64), (128, 32), (1000, 8), (10000, 2)]:
        for coalesce in ([False, True] if nq < 10000 else [False]):
            r = run(nq, threads, coalesce)
            print(r, file=sys.stderr, flush=True)
            out.append(r)
    print(json.dumps({"index": f"IVF_FLAT d=128 N={args.n} nlist={args.nlist} nprobe={args.nprobe} k=10",
                      "max_batch": args.max_batch, "wait_us": args.wait_us,
                      "client": "Python threads over ctypes (pyr_index_search, host buffers, PCIe-inclusive)",
                      "results": out}))


if __name__ == "__main__":
    main()
