"""Every dimension on the stream scan.

The round-4 scan (scan.hip) pads the fp16 tiles and query operands to a tile dimension (dims up to 128
rounded up to 32, then 256 / 512 / 768) with zeros; the fp32 rows, the exact refine and the re-run keep
the real dimension, with the reference's remainder loops for d % 8 != 0 (VectorMath.cs:229-250 and the
8-lane loops' tails).  Each case checks the stream path ran (the profiler's sample phase) and that the
ids and score bits equal the oracle's: FLAT L2 / IP / Cosine (BruteForceVectorIndex.cs:350-356, the
*Unsafe forms) and IVF_FLAT L2 / IP / Cosine (IvfFlatVectorIndex.cs:351-360, the safe forms).
"""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

DIMS = [96, 100, 200, 256, 768]
K = 10


def _sampled(lib, run):
    """run() with the profiler on; returns its result and the sample phase's call count (stream scan)"""
    lib.pyr_profile_reset()
    lib.pyr_profile_enable(1)
    try:
        out = run()
    finally:
        lib.pyr_profile_enable(0)
    ms, calls, work = C.c_double(), C.c_int64(), C.c_int64()
    lib.pyr_profile_get(9, C.byref(ms), C.byref(calls), C.byref(work))
    return out, calls.value


def _same(s, l, os_, ok):
    np.testing.assert_array_equal(l, ok)
    assert np.array_equal(s.view(np.uint32), os_.astype(np.float32).view(np.uint32))


@pytest.mark.parametrize("metric", [0, 1, 2])
@pytest.mark.parametrize("dim", DIMS)
def test_flat_dims_match_oracle(hiplib, oracle, dim, metric):
    from pyrope_amd import BruteForceVectorIndex, generate_synthetic
    n = 12000 if dim <= 256 else 6000  # FLAT chunks of 10,240 rows: two "lists" at the smaller dims
    x = generate_synthetic(n, dim, 42)
    q = generate_synthetic(24, dim, 1337)
    idx = BruteForceVectorIndex(dim, metric)
    idx.add_labels(np.arange(n, dtype=np.int64), x)
    (s, l, c), calls = _sampled(hiplib, lambda: idx.search_batch(q, K))
    assert calls >= 1, "the FLAT search must take the stream scan"
    for i in range(len(q)):
        os_, ok = oracle.bf_search(x, None, metric, q[i], K)
        _same(s[i], l[i], os_, ok)


@pytest.mark.parametrize("metric", [0, 1, 2])
@pytest.mark.parametrize("dim", DIMS)
def test_ivf_dims_match_oracle(hiplib, oracle, dim, metric):
    from pyrope_amd import IvfFlatVectorIndex, SearchOptions, generate_synthetic
    n = 8192 if dim <= 256 else 4096
    x = generate_synthetic(n, dim, 42)
    q = generate_synthetic(24, dim, 1337)
    idx = IvfFlatVectorIndex(dim, metric, n_list=32)
    idx.add_labels(np.arange(n, dtype=np.int64), x)
    idx.build()
    opts = SearchOptions(nprobe=8)
    (s, l, c), calls = _sampled(hiplib, lambda: idx.search_batch(q, K, opts))
    assert calls >= 1, "the IVF search must take the stream scan"
    off, labels, live = idx.ivf_layout()
    rows = x[np.where(labels >= 0, labels, 0)]
    cents = idx.centroids_array()
    for i in range(len(q)):
        os_, ok = oracle.ivf_search(q[i], K, cents, rows, off, live, metric=metric, nprobe=8)
        _same(s[i], l[i], os_, labels[ok])


@pytest.mark.parametrize("dim", [96, 128])
def test_flat_many_queries_per_item(hiplib, oracle, dim):
    """600 queries: items of 512 query slots (more than one item per chunk), the tile loop over 16 groups"""
    from pyrope_amd import BruteForceVectorIndex, generate_synthetic
    n = 20000
    x = generate_synthetic(n, dim, 42)
    q = generate_synthetic(600, dim, 7)
    idx = BruteForceVectorIndex(dim, 0)
    idx.add_labels(np.arange(n, dtype=np.int64), x)
    (s, l, c), calls = _sampled(hiplib, lambda: idx.search_batch(q, K))
    assert calls >= 1
    for i in range(0, len(q), 37):
        os_, ok = oracle.bf_search(x, None, 0, q[i], K)
        _same(s[i], l[i], os_, ok)
