#!/usr/bin/env python3
"""Latency of small IVF batches on the I1 index (d=128 N=10M nlist=1024 nprobe=32 k=10).

For nq in --sizes: HBM-resident queries, pyr_index_search_device on one stream, the mean time per
batch over --reps batches (host clock around a synchronised loop) and the per-phase HIP-event times
(pyr_profile_*).  This is the floor a coalesced serving batch pays (Serving).  JSON on stdout.

    python scripts/small_batch.py > profiles/r3_aux/small_batch.json
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PH = {0: "coarse", 1: "work_lists", 2: "list_scan", 4: "merge", 7: "refine", 8: "exact_rerun", 9: "sample"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=10_000_000)
    ap.add_argument("--nlist", type=int, default=1024)
    ap.add_argument("--nprobe", type=int, default=32)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--sizes", default="1,8,64,256,1024,4096")
    args = ap.parse_args()
    import torch
    torch.cuda.init()
    from pyrope_amd import IvfFlatVectorIndex, VectorMetric, _lib, generate_synthetic, generate_synthetic_blocked
    from pyrope_amd import kmeans_train
    from pyrope_amd.vector import SearchOptions
    L = _lib.load()
    D, k = 128, 10
    x = generate_synthetic_blocked(0, args.n, D, 42)
    cents = kmeans_train(x, args.nlist, VectorMetric.L2, 10, 42)
    idx = IvfFlatVectorIndex(D, VectorMetric.L2, n_list=args.nlist)
    idx.set_centroids(cents)
    idx.add_labels(np.arange(args.n, dtype=np.int64), x, track_ids=False)
    idx.build()
    del x
    qh = generate_synthetic(max(int(s) for s in args.sizes.split(",")), D, 1337)
    q = torch.from_numpy(qh).cuda()
    opts = SearchOptions(nprobe=args.nprobe)
    st = torch.cuda.current_stream().cuda_stream
    out = []
    for nq in [int(s) for s in args.sizes.split(",")]:
        s = torch.empty((nq, k), dtype=torch.float32, device="cuda")
        lab = torch.empty((nq, k), dtype=torch.int64, device="cuda")

        def run():
            idx.search_device(q.data_ptr(), nq, k, s.data_ptr(), lab.data_ptr(), 0, st, opts)
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(args.reps):
            run()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t) / args.reps * 1e3
        L.pyr_profile_reset()
        L.pyr_profile_enable(1)
        for _ in range(5):
            run()
        torch.cuda.synchronize()
        L.pyr_profile_enable(0)
        ph = {}
        for i, name in PH.items():
            m, c, w = C.c_double(), C.c_int64(), C.c_int64()
            L.pyr_profile_get(i, C.byref(m), C.byref(c), C.byref(w))
            if c.value:
                ph[name] = round(m.value / 5, 4)
        r = {"nq": nq, "ms_per_batch": ms, "qps": nq / ms * 1e3, "phases_ms": ph}
        print(r, file=sys.stderr, flush=True)
        out.append(r)
    print(json.dumps({"index": f"IVF_FLAT d=128 N={args.n} nlist={args.nlist} nprobe={args.nprobe} k=10",
                      "note": "HBM-resident queries, search_device back to back on one stream", "results": out}))


if __name__ == "__main__":
    main()
