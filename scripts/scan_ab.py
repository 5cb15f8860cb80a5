#!/usr/bin/env python3
"""A/B of measurement-only variants on the I1 index (IVF_FLAT d=128 N=10M nlist=1024 nprobe=32 k=10), 10,000
HBM-resident queries: per variant (a set of environment knobs, honoured with PYR_DEV_KNOBS=1) the step time
(median of --reps HIP-event-timed searches), the library's per-phase times (pyr_profile_*) and whether the
answers equal the default's bit for bit.  One JSON line on stdout.

    PYR_DEV_KNOBS=1 python scripts/scan_ab.py --variants 'base:;prio:PYR_FILTER_ABLATE=4096'
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


def parse(spec):
    out = []
    for part in spec.split(";"):
        if not part.strip():
            continue
        name, _, kv = part.partition(":")
        env = {}
        for a in kv.split(","):
            if a.strip():
                k, _, v = a.partition("=")
                env[k.strip()] = v.strip()
        out.append((name.strip(), env))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=10_000_000)
    ap.add_argument("--nq", type=int, default=10_000)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=2, help="passes over the variant list (box clock drift)")
    ap.add_argument("--variants", default="base:")
    args = ap.parse_args()
    import torch
    torch.cuda.init()
    from pyrope_amd import IvfFlatVectorIndex, SearchOptions, _lib, generate_synthetic, generate_synthetic_blocked
    from pyrope_amd import kmeans_train
    L = _lib.load()
    D = 128
    t0 = time.time()
    x = generate_synthetic_blocked(0, args.n, D, 42)
    cents = kmeans_train(x, 1024, 0, 10, 42)
    idx = IvfFlatVectorIndex(D, 0, n_list=1024)
    idx.set_centroids(cents)
    idx.add_labels(np.arange(args.n, dtype=np.int64), x, track_ids=False)
    idx.build()
    del x
    print(f"[scan_ab] built in {time.time() - t0:.1f}s", file=sys.stderr, flush=True)
    q = torch.from_numpy(generate_synthetic(args.nq, D, 1337)).cuda()
    opts = SearchOptions(nprobe=32)
    st = torch.cuda.current_stream()
    s = torch.empty((args.nq, args.k), dtype=torch.float32, device="cuda")
    lab = torch.empty((args.nq, args.k), dtype=torch.int64, device="cuda")

    def run():
        idx.search_device(q.data_ptr(), args.nq, args.k, s.data_ptr(), lab.data_ptr(), 0, st.cuda_stream, opts)

    variants = parse(args.variants)
    res = {"index": f"IVF_FLAT d=128 N={args.n} nlist=1024 nprobe=32 k={args.k}", "nq": args.nq, "variants": {}}
    ref = None
    for rnd in range(args.rounds):
        for name, env in variants:
            old = {k: os.environ.get(k) for k in env}
            os.environ.update(env)
            try:
                for _ in range(3):
                    run()
                torch.cuda.synchronize()
                ts = []
                for _ in range(args.reps):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(st)
                    run()
                    e1.record(st)
                    torch.cuda.synchronize()
                    ts.append(e0.elapsed_time(e1))
                out = (s.cpu().numpy().view(np.uint32).copy(), lab.cpu().numpy().copy())
                L.pyr_profile_reset()
                L.pyr_profile_enable(1)
                run()
                torch.cuda.synchronize()
                L.pyr_profile_enable(0)
            finally:
                for k, v in old.items():
                    if v is None:
                        os.environ.pop(k, None)
                    else:
                        os.environ[k] = v
            ph = {}
            for i, pn in PH.items():
                m_, c_, w_ = C.c_double(), C.c_int64(), C.c_int64()
                L.pyr_profile_get(i, C.byref(m_), C.byref(c_), C.byref(w_))
                if c_.value:
                    ph[pn] = round(m_.value, 4)
            if ref is None:
                ref = out
            same = bool(np.array_equal(out[0], ref[0]) and np.array_equal(out[1], ref[1]))
            r = res["variants"].setdefault(name, {"env": env, "ms": [], "phases_ms": [], "identical": []})
            r["ms"].append(round(float(np.median(ts)), 4))
            r["phases_ms"].append(ph)
            r["identical"].append(same)
            print(f"[scan_ab] round {rnd} {name}: {np.median(ts):.4f} ms (min {np.min(ts):.4f}), identical {same}, "
                  f"{ph}", file=sys.stderr, flush=True)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
