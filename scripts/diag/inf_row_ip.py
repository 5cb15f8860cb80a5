"""Diagnostic: FLAT IP with one +Inf element -- filter path vs exact scan vs oracle."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: F401
from pyrope_amd import BruteForceVectorIndex, generate_synthetic
import oracle

d = 128
x = generate_synthetic(20000, d, 42)
x[5000] = np.nan
x[7000, 3] = np.inf
q = generate_synthetic(200, d, 1337)
idx = BruteForceVectorIndex(d, 1)
idx.add_labels(np.arange(len(x), dtype=np.int64), x)
s1, l1, c1 = idx.search_batch(q, 10)
os.environ["PYR_FILTER"] = "0"
s2, l2, c2 = idx.search_batch(q, 10)
os.environ.pop("PYR_FILTER")
bad = [i for i in range(len(q)) if not np.array_equal(l1[i], l2[i])]
print("mismatching queries", len(bad), bad[:10])
for i in bad[:3]:
    os_, ol = oracle.bf_search(x, None, 1, q[i], 10)
    print("q", i)
    print(" filter", l1[i].tolist(), s1[i].tolist())
    print(" exact ", l2[i].tolist(), s2[i].tolist())
    print(" oracle", ol.tolist(), os_.tolist())
