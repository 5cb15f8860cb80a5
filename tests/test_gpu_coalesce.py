"""Request coalescing (pyr_index_set_coalescing): concurrent single-query searches -- the
reference's one index.Search per VEC.SEARCH (Extensions/VectorCommandSet.cs:457-459) from many
session threads -- are merged into device batches; every caller must get exactly what a search
of its queries alone returns."""
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _same(a, b):
    (s1, l1, c1), (s2, l2, c2) = a, b
    np.testing.assert_array_equal(c1, c2)
    np.testing.assert_array_equal(l1, l2)
    assert np.array_equal(s1.view(np.uint32), s2.view(np.uint32))


@pytest.mark.parametrize("kind", ["ivf", "flat"])
def test_concurrent_coalesced_searches_equal_sequential(hiplib, kind):
    from pyrope_amd import BruteForceVectorIndex, IvfFlatVectorIndex, SearchOptions, generate_synthetic
    x = generate_synthetic(50_000, 64, 21)
    q = generate_synthetic(1200, 64, 22)
    if kind == "ivf":
        idx = IvfFlatVectorIndex(64, 0, n_list=32)
        idx.add_labels(np.arange(len(x), dtype=np.int64), x)
        idx.build()
    else:
        idx = BruteForceVectorIndex(64, 1)
        idx.add_labels(np.arange(len(x), dtype=np.int64), x)
    # per-call shapes: (first query, count, k, options) -- keys that must not be merged together
    calls = []
    rng = np.random.default_rng(3)
    i = 0
    while i < len(q):
        n = int(rng.choice([1, 1, 1, 2, 5, 17]))
        k = int(rng.choice([10, 10, 3]))
        opts = SearchOptions(nprobe=int(rng.choice([4, 8]))) if kind == "ivf" else None
        calls.append((i, min(n, len(q) - i), k, opts))
        i += n
    ref = [idx.search_batch(q[a:a + n], k, o) for a, n, k, o in calls]
    idx.set_coalescing(256, 3000)
    got = [None] * len(calls)
    errors = []

    def worker(t):
        try:
            for j in range(t, len(calls), 24):
                a, n, k, o = calls[j]
                got[j] = idx.search_batch(q[a:a + n], k, o)
        except Exception as e:  # noqa: BLE001 -- surfaced below
            errors.append(e)

    th = [threading.Thread(target=worker, args=(t,)) for t in range(24)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors
    for r, g in zip(ref, got):
        _same(r, g)
    idx.set_coalescing(0, 0)
    _same(ref[0], idx.search_batch(q[:calls[0][1]], calls[0][2], calls[0][3]))
