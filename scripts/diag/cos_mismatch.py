"""Diagnostic: the cosine FLAT filter path vs the exact scan after upserts + deletes
(tests/test_gpu_cosine.py::test_cosine_writes_deletes_maxscans_snapshot), under env toggles."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def run(env):
    from pyrope_amd import BruteForceVectorIndex, SearchOptions, generate_synthetic
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        dim = 128
        x = generate_synthetic(8000, dim, 3)
        q = generate_synthetic(100, dim, 4)
        idx = BruteForceVectorIndex(dim, 2)
        idx.add_batch([f"v{i}" for i in range(len(x))], x)
        up = generate_synthetic(6, dim, 11)
        idx.upsert_batch(["v5", "new1", "v5", "v9", "new2", "new1"], up)
        for i in range(0, 8000, 97):
            idx.delete(f"v{i}")
        out = []
        for opts in (None, SearchOptions(max_scans=3000)):
            got = idx.search_batch(q, 10, opts)
            os.environ["PYR_FILTER"] = "0"
            ref = idx.search_batch(q, 10, opts)
            os.environ.pop("PYR_FILTER")
            bad = np.nonzero((got[1] != ref[1]).any(1))[0]
            out.append(len(bad))
            for b in bad[:3]:
                print("  query", b, "filter", got[1][b].tolist(), got[0][b].view(np.uint32).tolist())
                print("  query", b, "exact ", ref[1][b].tolist(), ref[0][b].view(np.uint32).tolist())
        idx.close()
        return out
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


for env in ({}, {"PYR_MERGE_REFINE": "0"}, {"PYR_SMALL_WRITE": "0"}, {"PYR_STREAM_DEBUG": "1"}):
    print(env, "mismatched queries (no MaxScans, MaxScans 3000):", run(env), flush=True)
