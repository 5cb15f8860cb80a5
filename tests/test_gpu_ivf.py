"""IVF_FLAT on the GPU vs the CPU oracle.

Build (KMeansUtils.Train seed 42 + FindNearestCentroid) must give bit-identical
centroids and the same list layout; Search must give the oracle's ids and
bit-identical scores.  Reference: Vector/IvfFlatVectorIndex.cs, Vector/KMeansUtils.cs,
tests/.../IvfFlatVectorIndexTests.cs.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _build(dim, metric, n, nlist, seed=42):
    from pyrope_amd import IvfFlatVectorIndex, generate_synthetic
    x = generate_synthetic(n, dim, seed)
    idx = IvfFlatVectorIndex(dim, metric, n_list=nlist)
    idx.add_labels(np.arange(n, dtype=np.int64), x)
    idx.build()
    return idx, x


def _oracle_layout(idx, x):
    off, labels, live = idx.ivf_layout()
    rows = x[np.where(labels >= 0, labels, 0)]
    return off, labels, live, rows


def _same(gs, gl, gc, os_, ok, labels_of_key):
    assert int(gc) == len(os_), (gc, len(os_))
    exp = np.array([labels_of_key(k) for k in ok], np.int64)
    np.testing.assert_array_equal(gl[: len(exp)], exp)
    assert np.array_equal(gs[: len(os_)].view(np.uint32), os_.astype(np.float32).view(np.uint32))


@pytest.mark.parametrize("metric", [0, 1, 2])
def test_ivf_build_matches_oracle(hiplib, oracle, metric):
    idx, x = _build(128, metric, 8192, 64)
    cents, assign = oracle.ivf_build(x, 64, metric)
    g = idx.centroids_array()
    assert g.shape == cents.shape
    assert np.array_equal(g.view(np.uint32), cents.view(np.uint32))
    off, labels, live = idx.ivf_layout()
    _, order, ooff = oracle.lists_from_assign(x, assign, len(cents))
    np.testing.assert_array_equal(off, ooff)
    np.testing.assert_array_equal(labels, order)


@pytest.mark.parametrize("metric", [0, 1, 2])
@pytest.mark.parametrize("nprobe", [1, 8, 64])
def test_ivf_search_matches_oracle(hiplib, oracle, metric, nprobe):
    from pyrope_amd import SearchOptions, generate_synthetic
    idx, x = _build(128, metric, 8192, 64)
    off, labels, live, rows = _oracle_layout(idx, x)
    cents = idx.centroids_array()
    q = generate_synthetic(40, 128, 1337)
    s, l, c = idx.search_batch(q, 10, SearchOptions(nprobe=nprobe))
    for i in range(len(q)):
        os_, ok = oracle.ivf_search(q[i], 10, cents, rows, off, live, metric=metric, nprobe=nprobe)
        _same(s[i], l[i], c[i], os_, ok, lambda k: labels[k])


@pytest.mark.parametrize("dim", [64, 96, 32, 20])
def test_ivf_other_dims(hiplib, oracle, dim):
    from pyrope_amd import SearchOptions, generate_synthetic
    idx, x = _build(dim, 0, 3000, 16)
    cents, assign = oracle.ivf_build(x, 16, 0)
    assert np.array_equal(idx.centroids_array().view(np.uint32), cents.view(np.uint32))
    off, labels, live, rows = _oracle_layout(idx, x)
    q = generate_synthetic(16, dim, 5)
    s, l, c = idx.search_batch(q, 10, SearchOptions(nprobe=4))
    for i in range(len(q)):
        os_, ok = oracle.ivf_search(q[i], 10, cents, rows, off, live, nprobe=4)
        _same(s[i], l[i], c[i], os_, ok, lambda k: labels[k])


def test_ivf_buffer_shadow_delete_and_max_scans(hiplib, oracle):
    """Rows added after Build live in the exact-scanned buffer; list rows with a buffered id are skipped
    (IvfFlatVectorIndex.cs:170-180, :210); Delete removes from both (:61-83); MaxScans counts both (:172,:202-212)."""
    from pyrope_amd import SearchOptions, generate_synthetic
    idx, x = _build(128, 0, 6000, 32)
    extra = generate_synthetic(300, 128, 777)
    # 200 new ids + 100 overwrites of existing ids (shadowing their list rows)
    new_labels = np.concatenate([np.arange(6000, 6200), np.arange(0, 100)])
    idx.add_labels(new_labels, extra)
    for d in [3, 150, 6010, 4000]:
        assert idx.delete(str(d))
    buf_labels = [l for l in new_labels.tolist() if l not in (3, 150, 6010)]
    buf_rows = np.stack([extra[new_labels.tolist().index(l)] for l in buf_labels])
    # Dictionary slot order: deleted slots are free; no insertion after them, so order = insertion minus deleted
    off, labels, live, rows = _oracle_layout(idx, x)
    cents = idx.centroids_array()
    q = generate_synthetic(24, 128, 4242)
    for ms in [None, 0, 150, 297, 900, 5000]:
        opts = SearchOptions(nprobe=5, max_scans=ms)
        s, l, c = idx.search_batch(q, 10, opts)
        for i in range(len(q)):
            # oracle buffer keeps the GPU's slot order: all 300 slots with 3 freed
            slot_labels = new_labels.tolist()
            bl = np.array([lab not in (3, 150, 6010) for lab in slot_labels], np.uint8)
            os_, ok = oracle.ivf_search(q[i], 10, cents, rows, off, live, buf=extra, buf_live=bl, nprobe=5,
                                        max_scans=-1 if ms is None else ms)

            def lab_of(k):
                return slot_labels[k - oracle.BUFKEY] if k >= oracle.BUFKEY else labels[k]
            _same(s[i], l[i], c[i], os_, ok, lab_of)
    assert len(buf_labels) == 298
    assert idx.get_stats().count == 298 + 6000 - 3  # buffer + list rows (shadowed counted, :305)


def test_ivf_rebuild_merges_buffer(hiplib, oracle):
    """Build after adds: uniqueData = list rows (buffer value wins) then new buffer ids (:90-113)."""
    from pyrope_amd import generate_synthetic
    idx, x = _build(128, 0, 3000, 16)
    off, labels, live = idx.ivf_layout()
    extra = generate_synthetic(50, 128, 9)
    new_labels = np.concatenate([np.arange(3000, 3025), np.arange(10, 35)])
    idx.add_labels(new_labels, extra)
    idx.build()
    # expected uniqueData order
    data = {int(l): x[l] for l in range(3000)}
    order = [int(lb) for lb in labels.tolist()]
    for lab, row in zip(new_labels.tolist(), extra):
        data[lab] = row
    for lab in new_labels.tolist():
        if lab not in order:
            order.append(lab)
    u = np.stack([data[lb] for lb in order])
    cents, assign = oracle.ivf_build(u, 16, 0)
    assert np.array_equal(idx.centroids_array().view(np.uint32), cents.view(np.uint32))
    off2, labels2, _ = idx.ivf_layout()
    _, perm, ooff = oracle.lists_from_assign(u, assign, len(cents))
    np.testing.assert_array_equal(labels2, np.array(order)[perm])


# ---- IvfFlatVectorIndexTests.cs ----
def test_get_centroids_before_build_returns_null(hiplib):
    from pyrope_amd import IvfFlatVectorIndex, VectorMetric
    index = IvfFlatVectorIndex(2, VectorMetric.L2, n_list=2)
    index.add("a", [1.0, 0.0])
    assert index.get_centroids() is None


def test_get_centroids_after_build_returns_list(hiplib):
    from pyrope_amd import IvfFlatVectorIndex, VectorMetric
    index = IvfFlatVectorIndex(2, VectorMetric.L2, n_list=2)
    for i, v in [("a1", [0.1, 0.1]), ("a2", [0.2, 0.2]), ("b1", [10.1, 10.1]), ("b2", [10.2, 10.2])]:
        index.add(i, v)
    index.build()
    c = index.get_centroids()
    assert c is not None and len(c) == 2 and all(len(r) == 2 for r in c)


def test_search_before_build_returns_results_from_buffer(hiplib):
    from pyrope_amd import IvfFlatVectorIndex, VectorMetric
    index = IvfFlatVectorIndex(2, VectorMetric.L2, n_list=2)
    index.add("a", [1.0, 0.0])
    index.add("b", [5.0, 5.0])
    r = index.search([1.0, 0.0], 1)
    assert len(r) == 1 and r[0].id == "a"


def test_build_clusters_data(hiplib):
    from pyrope_amd import IvfFlatVectorIndex, SearchOptions, VectorMetric
    index = IvfFlatVectorIndex(2, VectorMetric.L2, n_list=2)
    for i, v in [("a1", [0.1, 0.1]), ("a2", [0.2, 0.2]), ("b1", [10.1, 10.1]), ("b2", [10.2, 10.2])]:
        index.add(i, v)
    index.build()
    r = index.search([0.0, 0.0], 2, SearchOptions(max_scans=None))
    assert len(r) == 2
    assert any(x.id.startswith("a") for x in r)


def test_search_with_nprobe_increases_recall(hiplib):
    from pyrope_amd import IvfFlatVectorIndex, VectorMetric
    index = IvfFlatVectorIndex(2, VectorMetric.L2, n_list=3)
    index.combine_nprobe = 1
    index.add("c1", [0.0, 0.0])
    index.add("c2", [5.0, 5.0])
    index.add("c3", [10.0, 10.0])
    index.build()
    index.combine_nprobe = 3
    assert len(index.search([0.0, 0.0], 3)) == 3


def test_concurrent_searches_match_sequential(hiplib):
    """The reference serves Search from many session threads at once under a read lock
    (IvfFlatVectorIndex.cs ReaderWriterLockSlim); the C ABI allows concurrent pyr_index_search
    calls (a workspace per call).  Results under contention equal the sequential ones."""
    import threading

    from pyrope_amd import IvfFlatVectorIndex, SearchOptions, generate_synthetic
    x = generate_synthetic(30000, 64, 21)
    idx = IvfFlatVectorIndex(64, 0, n_list=32)
    idx.add_labels(np.arange(len(x), dtype=np.int64), x)
    idx.build()
    qs = [generate_synthetic(50, 64, 100 + t) for t in range(8)]
    opts = SearchOptions(nprobe=6)
    ref = [idx.search_batch(q, 10, opts) for q in qs]
    got = [None] * len(qs)
    errors = []

    def run(t):
        try:
            for _ in range(5):
                got[t] = idx.search_batch(qs[t], 10, opts)
        except Exception as e:  # surfaced below
            errors.append(e)

    th = [threading.Thread(target=run, args=(t,)) for t in range(len(qs))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors
    for r, g in zip(ref, got):
        np.testing.assert_array_equal(r[1], g[1])
        assert np.array_equal(r[0].view(np.uint32), g[0].view(np.uint32))
