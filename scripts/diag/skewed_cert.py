"""Diagnostic: certificate failures of the default fp16 stream path on the clustered-with-outliers
data of tests/test_gpu_ivf_chunks.py::test_per_list_certificate_on_skewed_data (PYR_STREAM_DEBUG
prints the candidate pool and the failing queries' margins)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from pyrope_amd import IvfFlatVectorIndex, SearchOptions  # noqa: E402


def clustered(n, nclu, d, seed, outliers):
    rng = np.random.default_rng(seed)
    centers = rng.standard_normal((nclu, d)).astype(np.float32) * 4
    lab = rng.integers(0, nclu, n)
    x = (centers[lab] + rng.standard_normal((n, d)).astype(np.float32)).astype(np.float32)
    far = rng.choice(n, outliers, replace=False)
    x[far] *= 300.0
    q = (centers[rng.integers(0, nclu, 400)] + rng.standard_normal((400, d)).astype(np.float32)).astype(np.float32)
    return x, q


for metric in (0, 1):
    x, q = clustered(60_000, 64, 128, 3, int(os.environ.get("OUTLIERS", "6")))
    idx = IvfFlatVectorIndex(128, metric, n_list=64)
    idx.add_labels(np.arange(len(x), dtype=np.int64), x)
    idx.build()
    print(f"metric {metric}", flush=True)
    os.environ["PYR_STREAM_DEBUG"] = "1"
    idx.search_batch(q, 10, SearchOptions(nprobe=8))
    os.environ.pop("PYR_STREAM_DEBUG")
