#!/usr/bin/env python3
"""Diagnostic (GPU box): candidate pools and certificate failures of the stream list scan on the
clustered test workloads (tests/test_gpu_ivf_chunks.py skewed data, tests/test_gpu_rk.py clusters).
Prints the library's PYR_STREAM_DEBUG summary per search and the exact re-run counts."""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def clustered(n, nclu, d, seed, outliers, nq):
    rng = np.random.default_rng(seed)
    centers = rng.standard_normal((nclu, d)).astype(np.float32) * 4
    lab = rng.integers(0, nclu, n)
    x = (centers[lab] + rng.standard_normal((n, d)).astype(np.float32)).astype(np.float32)
    if outliers:
        far = rng.choice(n, outliers, replace=False)
        x[far] *= 300.0
    q = (centers[rng.integers(0, nclu, nq)] + rng.standard_normal((nq, d)).astype(np.float32)).astype(np.float32)
    return x, q


def main():
    from pyrope_amd import IvfFlatVectorIndex, SearchOptions, _lib
    L = _lib.load()
    os.environ["PYR_STREAM_DEBUG"] = "1"
    cases = [("skewed 60k/64 +6 outliers", clustered(60_000, 64, 128, 3, 6, 400), 64, 8),
             ("clusters 50k/32", clustered(50_000, 32, 128, 5, 0, 600), 32, 4)]
    for name, (x, q), nl, npb in cases:
        for metric in (0, 1):
            idx = IvfFlatVectorIndex(128, metric, n_list=nl)
            idx.add_labels(np.arange(len(x), dtype=np.int64), x)
            idx.build()
            for prec in ("3", "2"):
                os.environ["PYR_STREAM_PREC"] = prec
                L.pyr_profile_reset()
                L.pyr_profile_enable(1)
                idx.search_batch(q, 10, SearchOptions(nprobe=npb))
                L.pyr_profile_enable(0)
                ms, calls, work = C.c_double(), C.c_int64(), C.c_int64()
                L.pyr_profile_get(8, C.byref(ms), C.byref(calls), C.byref(work))
                print(f"{name} metric={metric} prec={prec}: exact re-runs {work.value}/{len(q)}", flush=True)
            idx.close()


if __name__ == "__main__":
    main()
