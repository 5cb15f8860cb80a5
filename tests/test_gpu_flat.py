"""FLAT (BruteForceVectorIndex) on the GPU vs the CPU oracle: bit-identical scores, exact ids.

Reference: src/Pyrope.GarnetServer/Vector/BruteForceVectorIndex.cs:275-379 and
tests/Pyrope.GarnetServer.Tests/Vector/BruteForceVectorIndexTests.cs.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _flat(dim, metric, n, seed=42):
    from pyrope_amd import BruteForceVectorIndex, generate_synthetic
    x = generate_synthetic(n, dim, seed)
    idx = BruteForceVectorIndex(dim, metric)
    idx.add_labels(np.arange(n, dtype=np.int64), x)
    return idx, x


def _check_same(gs, gl, gc, os_, ok):
    """GPU (scores, labels, count) == oracle (scores, keys) with keys == labels."""
    assert int(gc) == len(os_)
    np.testing.assert_array_equal(gl[: len(ok)], ok)
    assert np.array_equal(gs[: len(os_)].view(np.uint32), os_.astype(np.float32).view(np.uint32)), (gs, os_)


@pytest.mark.parametrize("metric", [0, 1, 2])
@pytest.mark.parametrize("dim", [128, 64, 96, 32, 37, 8, 3])
def test_flat_bit_exact(hiplib, oracle, metric, dim):
    n, nq, k = 2048, 32, 10
    idx, x = _flat(dim, metric, n)
    from pyrope_amd import generate_synthetic
    q = generate_synthetic(nq, dim, 1337)
    s, l, c = idx.search_batch(q, k)
    for i in range(nq):
        os_, ok = oracle.bf_search(x, None, metric, q[i], k)
        _check_same(s[i], l[i], c[i], os_, ok)


@pytest.mark.parametrize("k", [1, 7, 64, 65, 200])
def test_flat_k_values(hiplib, oracle, k):
    idx, x = _flat(128, 0, 3000)
    from pyrope_amd import generate_synthetic
    q = generate_synthetic(5, 128, 7)
    s, l, c = idx.search_batch(q, k)
    for i in range(len(q)):
        os_, ok = oracle.bf_search(x, None, 0, q[i], k)
        _check_same(s[i], l[i], c[i], os_, ok)


def test_flat_max_scans_and_deletes(hiplib, oracle):
    from pyrope_amd import SearchOptions, generate_synthetic
    idx, x = _flat(128, 0, 5000)
    dead = np.arange(0, 5000, 7)
    for d in dead:
        assert idx.delete(str(d))
    live = np.ones(5000, np.uint8)
    live[dead] = 0
    q = generate_synthetic(4, 128, 99)
    for ms in [0, 1, 9, 777, 4999, 10_000]:
        s, l, c = idx.search_batch(q, 10, SearchOptions(max_scans=ms))
        for i in range(len(q)):
            os_, ok = oracle.bf_search(x, live, 0, q[i], 10, ms)
            _check_same(s[i], l[i], c[i], os_, ok)


def test_flat_ties_lowest_slot_first(hiplib, oracle):
    from pyrope_amd import BruteForceVectorIndex
    idx = BruteForceVectorIndex(128, 0)
    base = np.ones((1, 128), np.float32)
    x = np.repeat(base, 40, axis=0)
    idx.add_labels(np.arange(40), x)
    s, l, c = idx.search_batch(base, 10)
    assert list(l[0]) == list(range(10))


# ---- BruteForceVectorIndexTests.cs ----
def test_search_with_cosine_metric_returns_closest_vector(hiplib):
    from pyrope_amd import BruteForceVectorIndex, VectorMetric
    index = BruteForceVectorIndex(2, VectorMetric.Cosine)
    index.add("a", [1.0, 0.0])
    index.add("b", [0.0, 1.0])
    results = index.search([1.0, 0.1], 1)
    assert len(results) == 1 and results[0].id == "a"


def test_upsert_overwrites_existing_vector(hiplib):
    from pyrope_amd import BruteForceVectorIndex, VectorMetric
    index = BruteForceVectorIndex(2, VectorMetric.InnerProduct)
    index.add("a", [1.0, 0.0])
    index.upsert("a", [0.0, 2.0])
    results = index.search([0.0, 1.0], 1)
    assert results[0].id == "a" and results[0].score > 1.0


def test_delete_removes_vector(hiplib):
    from pyrope_amd import BruteForceVectorIndex, VectorMetric
    index = BruteForceVectorIndex(2, VectorMetric.L2)
    index.add("a", [1.0, 1.0])
    assert index.delete("a")
    assert index.search([1.0, 1.0], 1) == []


def test_add_with_wrong_dimension_throws(hiplib):
    from pyrope_amd import ArgumentException, BruteForceVectorIndex, VectorMetric
    index = BruteForceVectorIndex(2, VectorMetric.L2)
    with pytest.raises(ArgumentException):
        index.add("a", [1.0])


def test_search_with_max_scans_zero_returns_empty(hiplib):
    from pyrope_amd import BruteForceVectorIndex, SearchOptions, VectorMetric
    index = BruteForceVectorIndex(2, VectorMetric.InnerProduct)
    index.add("a", [1.0, 0.0])
    index.add("b", [0.0, 1.0])
    assert index.search([1.0, 0.0], 1, SearchOptions(max_scans=0)) == []


def test_duplicate_add_and_bad_topk(hiplib):
    from pyrope_amd import (ArgumentOutOfRangeException, BruteForceVectorIndex, InvalidOperationException,
                            VectorMetric)
    index = BruteForceVectorIndex(2, VectorMetric.L2)
    index.add("a", [1.0, 0.0])
    with pytest.raises(InvalidOperationException):
        index.add("a", [0.0, 1.0])
    with pytest.raises(ArgumentOutOfRangeException):
        index.search([1.0, 0.0], 0)
    assert index.get_stats().count == 1


def test_flat_large_sample_property(hiplib, oracle):
    """BASELINE F2 shape (N=1M, d=128): a sample of queries is exactly the oracle's answer."""
    from pyrope_amd import generate_synthetic
    n = 1_000_000
    idx, x = _flat(128, 0, n)
    q = generate_synthetic(256, 128, 1337)
    s, l, c = idx.search_batch(q, 10)
    for i in range(0, 256, 51):
        os_, ok = oracle.bf_search(x, None, 0, q[i], 10)
        _check_same(s[i], l[i], c[i], os_, ok)
    # sortedness and uniqueness for every query
    assert np.all(np.diff(s, axis=1) <= 0)
    assert all(len(set(r)) == 10 for r in l.tolist())
