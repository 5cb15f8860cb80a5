#!/usr/bin/env python3
"""Where the time of a deep top-k search goes (k > 60: deep_refine_kernel, filter.hip) on the I1 index
(IVF_FLAT d=128 N=10M nlist=1024 nprobe=32), 10,000 HBM-resident queries: per k the step time (median of
--reps) and the library's per-phase HIP-event times (pyr_profile_*: coarse, work lists, sample, list scan,
refine, exact re-run).  One JSON line on stdout.

    PYR_DEV_KNOBS=1 python scripts/deepk_phases.py [--ks 10,100,200,256]
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

PH = {0: "coarse", 1: "work_lists", 9: "sample", 2: "list_scan", 7: "refine", 8: "exact_rerun"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=10_000_000)
    ap.add_argument("--nq", type=int, default=10_000)
    ap.add_argument("--ks", default="10,100,200,256")
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import torch
    torch.cuda.init()
    from pyrope_amd import IvfFlatVectorIndex, SearchOptions, _lib, generate_synthetic, generate_synthetic_blocked
    from pyrope_amd import kmeans_train
    L = _lib.load()
    D = 128
    x = generate_synthetic_blocked(0, args.n, D, 42)
    cents = kmeans_train(x, 1024, 0, 10, 42)
    idx = IvfFlatVectorIndex(D, 0, n_list=1024)
    idx.set_centroids(cents)
    idx.add_labels(np.arange(args.n, dtype=np.int64), x, track_ids=False)
    idx.build()
    del x
    q = torch.from_numpy(generate_synthetic(args.nq, D, 1337)).cuda()
    opts = SearchOptions(nprobe=32)
    st = torch.cuda.current_stream().cuda_stream
    out = {"index": f"IVF_FLAT d=128 N={args.n} nlist=1024 nprobe=32", "nq": args.nq, "k": {}}
    for k in [int(v) for v in args.ks.split(",")]:
        s = torch.empty((args.nq, k), dtype=torch.float32, device="cuda")
        lab = torch.empty((args.nq, k), dtype=torch.int64, device="cuda")

        def run():
            idx.search_device(q.data_ptr(), args.nq, k, s.data_ptr(), lab.data_ptr(), 0, st, opts)
        run()
        torch.cuda.synchronize()
        ts = []
        for _ in range(args.reps):
            t = time.perf_counter()
            run()
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t) * 1e3)
        L.pyr_profile_reset()
        L.pyr_profile_enable(1)
        run()
        torch.cuda.synchronize()
        L.pyr_profile_enable(0)
        ph = {}
        for i, name in PH.items():
            m_, c_, w_ = C.c_double(), C.c_int64(), C.c_int64()
            L.pyr_profile_get(i, C.byref(m_), C.byref(c_), C.byref(w_))
            if c_.value:
                ph[name] = round(m_.value, 4)
        out["k"][k] = {"ms": round(float(np.median(ts)), 4), "phases_ms": ph}
        print(f"[deepk] k {k}: {out['k'][k]}", file=sys.stderr, flush=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
