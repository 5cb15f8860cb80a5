#!/usr/bin/env python3
"""Lane-width sensitivity of the parity pin: the reference's fp32 sums follow .NET's
Vector<float> width -- 8 lanes on x64 AVX2 (the oracle's assumption) or 4 on Arm64 NEON (where the
reference's published numbers were taken) -- and only the tie-breaking of near-equal
scores can depend on it.  Runs both builds of the CPU restatement (oracle/liboracle.so W = 8,
oracle/liboracle_w4.so W = 4) on the same data and counts queries whose top-10 ids differ.

    python scripts/lane_width.py > profiles/r2_lane_width.json   (CPU only, a few minutes)
"""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def compare(a, b):
    (s1, k1, _), (s2, k2, _) = a, b
    ordered = int(sum(not np.array_equal(x, y) for x, y in zip(k1, k2)))
    sets = int(sum(set(x.tolist()) != set(y.tolist()) for x, y in zip(k1, k2)))
    ids = int(sum(len(set(x.tolist()) ^ set(y.tolist())) // 2 for x, y in zip(k1, k2)))
    bits = int((s1.view(np.uint32) != s2.view(np.uint32)).sum())
    return {"queries": len(k1), "top10_order_differs": ordered, "top10_set_differs": sets, "ids_swapped": ids,
            "scores_with_other_bits": bits, "scores": int(s1.size)}


def main():
    import oracle
    from oracle import oracle as O
    N, D, NQ, NLIST, NPROBE, K = 1_000_000, 128, 500, 256, 32, 10
    threads = os.cpu_count() or 1
    x = oracle.generate_vectors(N, D, 42)
    q = oracle.generate_vectors(NQ, D, 1337)
    libs = {"W8": oracle.lib(), "W4": oracle.lib_w4()}
    out = {"data": f"uniform [0,1) synthetic (Program.cs:251-263), N={N}, d={D}, {NQ} queries, k={K}"}
    t = time.time()
    cents = oracle.kmeans_train(x[:100_000], NLIST, oracle.L2, 10, 42)  # one shared quantizer (W = 8 training)
    cn = np.zeros(len(cents), np.float32)
    # assignment of all rows with the W = 8 arithmetic (the index both variants search)
    import ctypes as C
    asg = np.empty(N, np.int32)
    for i in range(N):
        asg[i] = oracle.lib().orc_find_nearest_centroid(O._p(x[i], C.c_float), O._p(cents, C.c_float),
                                                        O._p(cn, C.c_float), NLIST, D, oracle.L2)
    lrows, order, off = oracle.lists_from_assign(x, asg, NLIST)
    print(f"index built in {time.time() - t:.0f}s", file=sys.stderr, flush=True)
    for metric, mname in [(oracle.L2, "L2"), (oracle.IP, "InnerProduct")]:
        res = {}
        for name, L in libs.items():
            O._lib = L
            t = time.time()
            flat = oracle.bf_search_batch(q, K, x, metric=metric, nthreads=threads)  # *Unsafe (4 accumulators)
            ivf = oracle.ivf_search_batch(q, K, cents, lrows, off, metric=metric, nprobe=NPROBE, nthreads=threads)
            res[name] = (flat, ivf)
            print(f"{mname} {name}: {time.time() - t:.0f}s", file=sys.stderr, flush=True)
        O._lib = libs["W8"]
        out[mname] = {"FLAT (BruteForce, *Unsafe sums)": compare(res["W8"][0], res["W4"][0]),
                      f"IVF_FLAT nlist={NLIST} nprobe={NPROBE} (safe sums, coarse ranking included)":
                          compare(res["W8"][1], res["W4"][1])}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
