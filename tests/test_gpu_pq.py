"""IVF_PQ on the GPU vs the CPU oracle: reference-identical training (coarse k-means seed 123,
per-subspace k-means seed 42+m), encoding, LUT and ADC sums.
Reference: Vector/IvfPqVectorIndex.cs, Vector/ProductQuantizer.cs, tests/.../IvfPqVectorIndexTests.cs.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _build(dim, metric, n, nlist, m, k=256, seed=42):
    from pyrope_amd import IvfPqVectorIndex, generate_synthetic
    x = generate_synthetic(n, dim, seed)
    idx = IvfPqVectorIndex(dim, metric, m=m, k=k, n_list=nlist)
    idx.add_labels(np.arange(n, dtype=np.int64), x)
    idx.build()
    return idx, x


@pytest.mark.parametrize("metric", [0, 1, 2])
def test_pq_build_matches_oracle(hiplib, oracle, metric):
    idx, x = _build(64, metric, 4096, 32, 8)
    cents, assign, cb, codes = oracle.ivfpq_build(x, 32, 8, 256, metric)
    assert np.array_equal(idx.centroids_array().view(np.uint32), cents.view(np.uint32))
    gcb, gcodes, off, labels, live = idx.pq_state()
    assert gcb.shape == cb.shape
    assert np.array_equal(gcb.view(np.uint32), cb.view(np.uint32))
    _, perm, ooff = oracle.lists_from_assign(x, assign, len(cents))
    np.testing.assert_array_equal(off, ooff)
    np.testing.assert_array_equal(labels, perm)
    np.testing.assert_array_equal(gcodes, codes[perm])


@pytest.mark.parametrize("metric", [0, 1, 2])
@pytest.mark.parametrize("nprobe", [1, 4])
def test_pq_search_matches_oracle(hiplib, oracle, metric, nprobe):
    from pyrope_amd import SearchOptions, generate_synthetic
    idx, x = _build(64, metric, 4096, 32, 8)
    gcb, gcodes, off, labels, live = idx.pq_state()
    cents = idx.centroids_array()
    q = generate_synthetic(24, 64, 1337)
    s, l, c = idx.search_batch(q, 10, SearchOptions(nprobe=nprobe))
    for i in range(len(q)):
        os_, ok = oracle.ivfpq_search(q[i], 10, cents, gcodes, off, gcb, live, metric=metric, nprobe=nprobe)
        assert int(c[i]) == len(os_)
        np.testing.assert_array_equal(l[i][: len(ok)], labels[ok])
        assert np.array_equal(s[i][: len(os_)].view(np.uint32), os_.view(np.uint32))


def test_pq_buffer_seen_and_delete(hiplib, oracle):
    """Buffer rows scanned exactly; list entries whose id is buffered are skipped (:134,:170);
    Delete touches only the buffer (:51), so the list entry becomes visible again."""
    from pyrope_amd import SearchOptions, generate_synthetic
    idx, x = _build(64, 0, 4096, 32, 8)
    extra = generate_synthetic(20, 64, 5)
    new = np.concatenate([np.arange(4096, 4106), np.arange(0, 10)])
    idx.add_labels(new, extra)
    assert idx.delete("5")
    gcb, gcodes, off, labels, live = idx.pq_state()
    cents = idx.centroids_array()
    bl = np.array([lab != 5 for lab in new.tolist()], np.uint8)
    q = generate_synthetic(8, 64, 77)
    s, l, c = idx.search_batch(q, 10, SearchOptions(nprobe=3))
    for i in range(len(q)):
        os_, ok = oracle.ivfpq_search(q[i], 10, cents, gcodes, off, gcb, live, buf=extra, buf_live=bl, nprobe=3)
        exp = [new[k - oracle.BUFKEY] if k >= oracle.BUFKEY else labels[k] for k in ok]
        np.testing.assert_array_equal(l[i][: len(exp)], exp)
        assert np.array_equal(s[i][: len(os_)].view(np.uint32), os_.view(np.uint32))
    assert idx.get_stats().count == 0  # GetStats quirk (:230)


def test_pq_d768_m96(hiplib, oracle):
    """BASELINE P1 geometry (d=768, M=96 -> 8-dim subspaces, K=256) at small N."""
    from pyrope_amd import SearchOptions, generate_synthetic
    idx, x = _build(768, 0, 1024, 8, 96)
    cents, assign, cb, codes = oracle.ivfpq_build(x, 8, 96, 256, 0)
    gcb, gcodes, off, labels, live = idx.pq_state()
    assert np.array_equal(gcb.view(np.uint32), cb.view(np.uint32))
    q = generate_synthetic(4, 768, 3)
    s, l, c = idx.search_batch(q, 10, SearchOptions(nprobe=2))
    for i in range(len(q)):
        os_, ok = oracle.ivfpq_search(q[i], 10, cents, gcodes, off, gcb, live, nprobe=2)
        np.testing.assert_array_equal(l[i][: len(ok)], labels[ok])
        assert np.array_equal(s[i][: len(os_)].view(np.uint32), os_.view(np.uint32))


# ---- IvfPqVectorIndexTests.cs ----
def test_ivfpq_search_returns_results(hiplib, oracle):
    from pyrope_amd import IvfPqVectorIndex, VectorMetric
    index = IvfPqVectorIndex(128, VectorMetric.L2, m=16, k=256, n_list=4)
    rng = oracle.NetRandom(123)
    for i in range(100):
        index.add(str(i), [rng.next_double() for _ in range(128)])
    index.build()
    results = index.search([0.5] * 128, 5)
    assert len(results) == 5


class _env:
    def __init__(self, **kv):
        self.kv = {k: str(v) for k, v in kv.items()}

    def __enter__(self):
        import os
        self.old = {k: os.environ.get(k) for k in self.kv}
        os.environ.update(self.kv)

    def __exit__(self, *a):
        import os
        for k, v in self.old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def _same(a, b):
    np.testing.assert_array_equal(a[2], b[2])
    np.testing.assert_array_equal(a[1], b[1])
    assert np.array_equal(a[0].view(np.uint32), b[0].view(np.uint32))


@pytest.mark.parametrize("dim,m,ksub,k", [(64, 8, 256, 10), (96, 24, 256, 1), (128, 32, 64, 33),
                                          (48, 48, 16, 64), (64, 16, 256, 65), (768, 96, 256, 10)])
def test_pq_adc_equals_first_kernel_and_oracle(hiplib, oracle, dim, m, ksub, k):
    """pq_adc (default) vs the first-cut pq_scan (PYR_PQ_ADC=0) vs the oracle: M not a multiple
    of 16, ksub < 256, k = 1 / 64 / 65."""
    from pyrope_amd import SearchOptions, generate_synthetic
    n = 6000 if dim < 768 else 3000
    idx, x = _build(dim, 0, n, 12, m, k=ksub)
    q = generate_synthetic(70, dim, 99)
    opts = SearchOptions(nprobe=5)
    got = idx.search_batch(q, k, opts)
    with _env(PYR_PQ_ADC=0):
        ref = idx.search_batch(q, k, opts)
    _same(got, ref)
    with _env(PYR_GTHR=0):
        _same(idx.search_batch(q, k, opts), ref)
    cb, codes, off, labels, live = idx.pq_state()
    cents = idx.centroids_array()
    for i in range(0, len(q), 23):
        os_, ok = oracle.ivfpq_search(q[i], k, cents, codes, off, cb, live, metric=0, nprobe=5)
        np.testing.assert_array_equal(got[1][i][: len(ok)], labels[ok])
        assert np.array_equal(got[0][i][: len(ok)].view(np.uint32), os_.view(np.uint32))


def test_pq_adc_ties_and_deletes(hiplib, oracle):
    """Duplicated rows give exact score ties (lowest storage position first); Delete after Build
    leaves listed rows in place (IvfPqVectorIndex.cs:51 touches only the buffer); listed rows
    whose id is re-added to the buffer are skipped (:134, :170)."""
    from pyrope_amd import IvfPqVectorIndex, SearchOptions, generate_synthetic
    base = generate_synthetic(300, 32, 5)
    x = np.repeat(base, 12, axis=0)
    idx = IvfPqVectorIndex(32, 0, m=4, k=32, n_list=6)
    idx.add_labels(np.arange(len(x), dtype=np.int64), x)
    idx.build()
    q = generate_synthetic(40, 32, 6)
    opts = SearchOptions(nprobe=3)
    before = idx.search_batch(q, 20, opts)
    for i in range(0, len(x), 5):
        idx.delete(str(i))
    _same(idx.search_batch(q, 20, opts), before)
    shadow = np.arange(0, len(x), 5)
    idx.add_labels(shadow, x[shadow] + 100.0)  # far away: the shadowed ids drop out of the top-20
    got = idx.search_batch(q, 20, opts)
    with _env(PYR_PQ_ADC=0):
        ref = idx.search_batch(q, 20, opts)
    _same(got, ref)
    assert not np.any(np.isin(got[1], shadow))


@pytest.mark.parametrize("metric", [0, 1])
def test_pq_build_with_given_quantizers_streams_identically(hiplib, oracle, metric):
    """set_centroids + set_codebooks (the P1 bulk path, engine.cpp IvfPqIndex::build_given): the
    build only assigns and encodes, in chunks (forced to 700 rows here), and must give the same lists,
    codes and search results as the reference build that trained those quantizers."""
    import os
    from pyrope_amd import IvfPqVectorIndex, SearchOptions, generate_synthetic
    ref, x = _build(64, metric, 4096, 32, 8)
    cents = ref.centroids_array()
    cb, codes, off, labels, live = ref.pq_state()
    idx = IvfPqVectorIndex(64, metric, m=8, k=256, n_list=32)
    idx.set_centroids(cents)
    idx.set_codebooks(cb)
    idx.reserve(len(x))
    for a in range(0, len(x), 1000):  # bulk load in several calls
        idx.add_labels(np.arange(a, min(a + 1000, len(x)), dtype=np.int64), x[a:a + 1000])
    os.environ["PYR_PQ_BUILD_CHUNK"] = "700"
    try:
        idx.build()
    finally:
        os.environ.pop("PYR_PQ_BUILD_CHUNK", None)
    gcb, gcodes, goff, glabels, glive = idx.pq_state()
    assert np.array_equal(gcb.view(np.uint32), cb.view(np.uint32))
    np.testing.assert_array_equal(goff, off)
    np.testing.assert_array_equal(glabels, labels)
    np.testing.assert_array_equal(gcodes, codes)
    q = generate_synthetic(32, 64, 1337)
    opts = SearchOptions(nprobe=4)
    s1, l1, c1 = ref.search_batch(q, 10, opts)
    s2, l2, c2 = idx.search_batch(q, 10, opts)
    np.testing.assert_array_equal(l1, l2)
    assert np.array_equal(s1.view(np.uint32), s2.view(np.uint32))
    with pytest.raises(Exception):
        idx.set_codebooks(cb[:4])  # wrong subspace count


@pytest.mark.parametrize("dim,m,ksub,k", [(64, 16, 256, 65), (128, 16, 256, 100), (96, 12, 256, 256),
                                          (48, 48, 16, 200), (100, 10, 256, 128), (768, 96, 256, 150)])
def test_pq_adc_large_k_equals_first_kernel_and_oracle(hiplib, oracle, dim, m, ksub, k):
    """The LUT scan at 64 < k <= 256 (pq_adc4 with four list registers per lane, 512-thread blocks): the
    matrix-core scan off (PYR_PQ_MFMA=0), so the LUT kernels answer; vs the first-cut pq_scan and the oracle.
    dsub 4 / 8 / 1 / 10 (the last not on pq32 at all), ksub 16, M not a multiple of 8."""
    from pyrope_amd import SearchOptions, generate_synthetic
    n = 6000 if dim < 768 else 3000
    idx, x = _build(dim, 0, n, 12, m, k=ksub)
    q = generate_synthetic(70, dim, 99)
    opts = SearchOptions(nprobe=5)
    with _env(PYR_PQ_MFMA=0):
        got = idx.search_batch(q, k, opts)
        with _env(PYR_PQ_ADC=0):
            ref = idx.search_batch(q, k, opts)
        with _env(PYR_GTHR=0):
            _same(idx.search_batch(q, k, opts), ref)
    _same(got, ref)
    np.testing.assert_array_equal(got[2], ref[2])
    _same(idx.search_batch(q, k, opts), ref)  # the default path (pq32 + deep refine where it applies)
    cb, codes, off, labels, live = idx.pq_state()
    cents = idx.centroids_array()
    for i in range(0, len(q), 23):
        os_, ok = oracle.ivfpq_search(q[i], k, cents, codes, off, cb, live, metric=0, nprobe=5)
        np.testing.assert_array_equal(got[1][i][: len(ok)], labels[ok])
        assert np.array_equal(got[0][i][: len(ok)].view(np.uint32), os_.view(np.uint32))
