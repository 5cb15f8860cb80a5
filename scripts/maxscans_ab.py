"""IVF_FLAT search with a MaxScans budget at I1: the stream scan vs the exact VALU scan (VERDICT r4 missing #5).

The reference's SLO guardrail degrades a search to MaxScans = SloGuardrailsOptions.DegradedMaxScans (5,000 by
default, Services/SloGuardrails.cs:73, SloGuardrailsOptions.cs:20); IvfFlatVectorIndex.Search then stops after
that many live rows in probe order (:200-218).  This script builds the I1 index (d = 128, N = 10M, nlist = 1,024)
and times search_device on 10,000 resident queries at nprobe 32 for each budget, stream path (default) and
exact path (PYR_MAXSCANS_STREAM=0), checking that both answers are bit-identical.

    python scripts/maxscans_ab.py [--n 10000000 --budgets 5000,50000,200000]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=10_000_000)
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--nlist", type=int, default=1024)
    ap.add_argument("--nprobe", type=int, default=32)
    ap.add_argument("--nq", type=int, default=10_000)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--budgets", default="5000,50000,200000")
    ap.add_argument("--topk", default="", help="comma list of k > 60: the deep refine vs the exact scan "
                    "(PYR_DEEP_REFINE=0)")
    ap.add_argument("--buffer", type=int, default=0, help="then add this many rows after Build (the buffer; half "
                    "of them new ids, half shadowing list rows) and time the search with it, stream vs exact")
    args = ap.parse_args()
    import torch
    torch.cuda.init()
    from pyrope_amd import (IvfFlatVectorIndex, SearchOptions, assign, generate_synthetic,
                            generate_synthetic_blocked, kmeans_train)
    N, D, NL, P, K = args.n, args.dim, args.nlist, args.nprobe, args.k
    t = time.time()
    data = generate_synthetic_blocked(0, N, D, 42, 65536)
    cents = kmeans_train(data, NL, 0, 10, 42)
    idx = IvfFlatVectorIndex(D, 0, n_list=NL)
    idx.set_centroids(cents)
    idx.reserve(N)
    for i in range(0, N, 2_000_000):
        idx.add_labels(np.arange(i, min(N, i + 2_000_000), dtype=np.int64), data[i:i + 2_000_000], track_ids=False)
    idx.build()
    del data
    print(f"[maxscans] built I1 in {time.time() - t:.1f}s", flush=True)
    dev = torch.device("cuda", 0)
    q = torch.from_numpy(generate_synthetic(args.nq, D, 1337)).to(dev)
    st = torch.cuda.current_stream()

    def run(opts):
        s = torch.empty((args.nq, K), dtype=torch.float32, device=dev)
        lab = torch.empty((args.nq, K), dtype=torch.int64, device=dev)
        c = torch.empty(args.nq, dtype=torch.int32, device=dev)
        idx.search_device(q.data_ptr(), args.nq, K, s.data_ptr(), lab.data_ptr(), c.data_ptr(),
                          stream=st.cuda_stream, options=opts)
        return s, lab, c

    def timed(opts):
        for _ in range(2):
            out = run(opts)
        torch.cuda.synchronize()
        ts = []
        for _ in range(args.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            out = run(opts)
            e1.record(st)
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        return float(np.median(ts)), float(np.min(ts)), [t.cpu().numpy() for t in out]

    res = {"config": {"n": N, "dim": D, "nlist": NL, "nprobe": P, "k": K, "nq": args.nq}, "budgets": {}}
    ms_none, _, _ = timed(SearchOptions(nprobe=P))
    res["no_budget_ms"] = ms_none
    print(f"[maxscans] no budget: {ms_none:.3f} ms", flush=True)
    for b in [int(v) for v in args.budgets.split(",") if v]:
        opts = SearchOptions(nprobe=P, max_scans=b)
        ms_s, mn_s, out_s = timed(opts)
        os.environ["PYR_MAXSCANS_STREAM"] = "0"
        try:
            ms_e, mn_e, out_e = timed(opts)
        finally:
            os.environ.pop("PYR_MAXSCANS_STREAM", None)
        os.environ["PYR_STREAM_DEBUG"] = "1"  # the emission and certificate statistics, to stderr
        try:
            run(opts)
            torch.cuda.synchronize()
        finally:
            os.environ.pop("PYR_STREAM_DEBUG", None)
        same = (np.array_equal(out_s[1], out_e[1]) and np.array_equal(out_s[2], out_e[2]) and
                np.array_equal(out_s[0].view(np.uint32), out_e[0].view(np.uint32)))
        res["budgets"][b] = {"stream_ms": ms_s, "stream_min_ms": mn_s, "exact_ms": ms_e, "exact_min_ms": mn_e,
                             "speedup": ms_e / ms_s, "bit_identical": bool(same),
                             "mean_results": float(out_s[2].mean())}
        print(f"[maxscans] budget {b}: stream {ms_s:.3f} ms, exact {ms_e:.3f} ms, x{ms_e / ms_s:.1f}, "
              f"identical {same}", flush=True)
        if not same:
            bad = np.nonzero((out_s[1] != out_e[1]).any(1))[0]
            print(f"[maxscans]   {len(bad)} queries differ, first {bad[:5].tolist()}", flush=True)
    for kk in [int(v) for v in args.topk.split(",") if v]:  # k > 60: depth 128 / 256 (deep_refine_kernel)
        opts = SearchOptions(nprobe=P)
        sv = K
        K = kk
        try:
            ms_s, mn_s, out_s = timed(opts)
            os.environ["PYR_DEEP_REFINE"] = "0"
            try:
                ms_e, mn_e, out_e = timed(opts)
            finally:
                os.environ.pop("PYR_DEEP_REFINE", None)
            os.environ["PYR_STREAM_DEBUG"] = "1"
            try:
                run(opts)
                torch.cuda.synchronize()
            finally:
                os.environ.pop("PYR_STREAM_DEBUG", None)
        finally:
            K = sv
        same = (np.array_equal(out_s[1], out_e[1]) and np.array_equal(out_s[2], out_e[2]) and
                np.array_equal(out_s[0].view(np.uint32), out_e[0].view(np.uint32)))
        res.setdefault("topk", {})[str(kk)] = {"stream_ms": ms_s, "exact_ms": ms_e, "speedup": ms_e / ms_s,
                                               "bit_identical": bool(same)}
        print(f"[maxscans] k {kk}: stream {ms_s:.3f} ms, exact {ms_e:.3f} ms, x{ms_e / ms_s:.1f}, identical {same}",
              flush=True)
    if args.buffer > 0:  # IvfFlatVectorIndex.cs:169-180: the buffer scanned exactly beside the lists
        nb = args.buffer
        lab = np.concatenate([np.arange(N, N + nb - nb // 2), np.arange(0, N, max(1, N // (nb // 2 + 1)))[: nb // 2]])
        idx.add_labels(lab.astype(np.int64), generate_synthetic(len(lab), D, 99))
        for b in [None, 5000]:
            opts = SearchOptions(nprobe=P, max_scans=b)
            ms_s, mn_s, out_s = timed(opts)
            os.environ["PYR_IVF_BUFFER_STREAM"] = "0"
            try:
                ms_e, mn_e, out_e = timed(opts)
            finally:
                os.environ.pop("PYR_IVF_BUFFER_STREAM", None)
            same = (np.array_equal(out_s[1], out_e[1]) and np.array_equal(out_s[2], out_e[2]) and
                    np.array_equal(out_s[0].view(np.uint32), out_e[0].view(np.uint32)))
            res.setdefault("buffer", {})[str(b)] = {"buffer_rows": len(lab), "stream_ms": ms_s, "exact_ms": ms_e,
                                                     "speedup": ms_e / ms_s, "bit_identical": bool(same)}
            print(f"[maxscans] buffer {len(lab)} rows, budget {b}: stream {ms_s:.3f} ms, exact {ms_e:.3f} ms, "
                  f"x{ms_e / ms_s:.1f}, identical {same}", flush=True)
    print(json.dumps(res), flush=True)
    idx.close()


if __name__ == "__main__":
    main()
