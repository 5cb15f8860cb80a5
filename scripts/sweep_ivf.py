#!/usr/bin/env python3
"""Measurement sweep for the IVF-Flat list scan (run on the GPU box): builds the bench index
once, prints list-size statistics, then times the batched search under each setting of the
PYR_* knobs given on the command line (env values are read by the library per search).

    python scripts/sweep_ivf.py --n 10000000 PYR_IVF_CHUNK=1024,2048,4096

--data mixture: a Gaussian mixture instead of the uniform bench rows -- `--clusters`
centres ~ N(0, 1)^d, rows = centre + N(0, sigma^2)^d, a fraction `--outliers` of the rows scaled
by `--outlier-scale`, queries drawn from the same mixture (no outliers) -- to measure how often the
default fp16 certificate re-runs queries on data that clusters.  --metric ip uses DotProduct, --metric cos VectorMath.Cosine.
"""
from __future__ import annotations

import argparse
import ctypes as C
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def mixture(args):
    """Gaussian-mixture rows and queries (float32), generated in 1M-row blocks."""
    rng = np.random.default_rng(7)
    cen = rng.standard_normal((args.clusters, args.dim)).astype(np.float32)
    x = np.empty((args.n, args.dim), dtype=np.float32)
    for b in range(0, args.n, 1 << 20):
        e = min(args.n, b + (1 << 20))
        lab = rng.integers(0, args.clusters, e - b)
        x[b:e] = cen[lab] + args.sigma * rng.standard_normal((e - b, args.dim), dtype=np.float32)
    far = rng.choice(args.n, max(1, int(args.n * args.outliers)), replace=False)
    x[far] *= args.outlier_scale
    q = cen[rng.integers(0, args.clusters, args.nq)] + args.sigma * rng.standard_normal((args.nq, args.dim),
                                                                                         dtype=np.float32)
    return x, q.astype(np.float32)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=10_000_000)
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--nlist", type=int, default=1024)
    ap.add_argument("--nprobe", type=int, default=32)
    ap.add_argument("--nq", type=int, default=10_000)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--prof-steps", type=int, default=3, help="profiled searches averaged per setting")
    ap.add_argument("--data", choices=["uniform", "mixture"], default="uniform")
    ap.add_argument("--train-rows", type=int, default=10_000_000, help="k-means rows (bench.py: all of I1)")
    ap.add_argument("--metric", choices=["l2", "ip", "cos"], default="l2")
    ap.add_argument("--clusters", type=int, default=1000)
    ap.add_argument("--sigma", type=float, default=0.5)
    ap.add_argument("--outliers", type=float, default=1e-4)
    ap.add_argument("--outlier-scale", type=float, default=30.0)
    ap.add_argument("knobs", nargs="*", help="NAME=v1,v2,...")
    ap.add_argument("--cfg", action="append", default=[],
                    help="one setting 'NAME=v,NAME2=v2' (repeatable; run after the knob grid)")
    args = ap.parse_args()

    import torch
    from pyrope_amd import (IvfFlatVectorIndex, VectorMetric, generate_synthetic, generate_synthetic_blocked,
                            kmeans_train, _lib)
    from pyrope_amd.vector import SearchOptions
    L = _lib.load()
    dev = torch.device("cuda", 0)
    met = {"l2": VectorMetric.L2, "ip": VectorMetric.InnerProduct, "cos": VectorMetric.Cosine}[args.metric]
    if args.data == "uniform":
        x = generate_synthetic_blocked(0, args.n, args.dim, 42)  # bench.py's row-blocked base set
        qh = generate_synthetic(args.nq, args.dim, 1337)
    else:
        x, qh = mixture(args)
    cents = kmeans_train(x[: min(args.n, args.train_rows)], args.nlist, met, 10, 42)
    idx = IvfFlatVectorIndex(args.dim, met, n_list=args.nlist)
    idx.set_centroids(cents)
    idx.add_labels(np.arange(args.n, dtype=np.int64), x, track_ids=False)
    idx.build()
    off, _, _ = idx.ivf_layout()
    ln = np.diff(off)
    print(f"lists: n={len(ln)} mean={ln.mean():.0f} min={ln.min()} p50={np.median(ln):.0f} "
          f"p99={np.percentile(ln, 99):.0f} max={ln.max()}", flush=True)
    q = torch.from_numpy(qh).to(dev)
    s = torch.empty((args.nq, args.k), dtype=torch.float32, device=dev)
    lab = torch.empty((args.nq, args.k), dtype=torch.int64, device=dev)
    opts = SearchOptions(nprobe=args.nprobe)
    st = torch.cuda.current_stream().cuda_stream

    def run():
        idx.search_device(q.data_ptr(), args.nq, args.k, s.data_ptr(), lab.data_ptr(), 0, st, opts)

    settings = [{}]
    for kv in args.knobs:
        name, vals = kv.split("=", 1)
        settings = [dict(d, **{name: v}) for d in settings for v in vals.split(",")]
    for c in args.cfg:
        settings.append(dict(kv.split("=", 1) for kv in c.split(",") if kv))
    ref = None
    touched = set()
    for cfg in settings:
        for kname in touched - set(cfg):
            os.environ.pop(kname, None)
        for kname, v in cfg.items():
            os.environ[kname] = v
            touched.add(kname)
        run()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(args.steps):
            run()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / args.steps
        L.pyr_profile_reset()
        L.pyr_profile_enable(1)
        for _ in range(args.prof_steps):
            run()
        torch.cuda.synchronize()
        L.pyr_profile_enable(0)
        ph = {}
        for i, name in {0: "coarse", 1: "items", 9: "sample", 2: "scan", 3: "buf", 4: "merge", 7: "refine", 8: "rerun"}.items():
            ms, calls, work = C.c_double(), C.c_int64(), C.c_int64()
            L.pyr_profile_get(i, C.byref(ms), C.byref(calls), C.byref(work))
            if calls.value:
                ph[name] = round(ms.value / args.prof_steps, 4)
            if i == 8 and calls.value:
                ph["reran_queries"] = work.value
        res = (s.cpu().numpy().copy(), lab.cpu().numpy().copy())
        same = None
        if ref is None:
            ref = res
        else:
            same = bool(np.array_equal(ref[0].view(np.uint32), res[0].view(np.uint32)) and
                        np.array_equal(ref[1], res[1]))
        print(f"{cfg}: {dt * 1e3:.2f} ms/step  {args.nq / dt:,.0f} QPS  phases {ph}  same_as_first={same}",
              flush=True)


if __name__ == "__main__":
    main()
