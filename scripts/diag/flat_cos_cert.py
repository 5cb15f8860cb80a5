"""FLAT Cosine certificate failures on the stream scan vs the round-3 filter (measurement only).

python scripts/diag/flat_cos_cert.py  -> per (dim, k): exact re-runs of 300 queries on 20,000 rows,
stream path (default) and PYR_FLAT_STREAM=0; PYR_STREAM_DEBUG lines go to stderr.
"""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def reruns(L, run):
    L.pyr_profile_reset()
    L.pyr_profile_enable(1)
    run()
    L.pyr_profile_enable(0)
    ms, calls, work = C.c_double(), C.c_int64(), C.c_int64()
    L.pyr_profile_get(8, C.byref(ms), C.byref(calls), C.byref(work))
    return work.value


def main():
    import torch
    torch.cuda.init()
    from pyrope_amd import BruteForceVectorIndex, _lib, generate_synthetic
    L = _lib.load()
    for dim in (32, 64, 128):
        x = generate_synthetic(20000, dim, 42)
        q = generate_synthetic(300, dim, 1337)
        idx = BruteForceVectorIndex(dim, 2)
        idx.add_labels(np.arange(len(x), dtype=np.int64), x)
        for k in (1, 10, 20):
            out = {}
            for mode in ("1", "0"):
                os.environ["PYR_FLAT_STREAM"] = mode
                out[mode] = reruns(L, lambda: idx.search_batch(q, k))
            os.environ.pop("PYR_FLAT_STREAM")
            print(f"dim {dim} k {k}: reruns stream {out['1']}, round-3 filter {out['0']}", flush=True)
        idx.close()


if __name__ == "__main__":
    main()
