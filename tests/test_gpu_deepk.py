"""IVF_FLAT with k > 60 on the stream scan (VERDICT r4 missing #5).

The reference takes any topK (IvfFlatVectorIndex.cs:147-231).  For 60 < k <= 256 the stream scan's emitted rows
are merged and refined at depth K1 = 128 / 256 / 512, k <= 0.8 K1 (deep_refine_kernel, one block per query: a bitonic sort of the
rows and the floor placeholders in LDS, exact re-scores in the reference's order, the upper-bound certificate);
what fails goes to the exact VALU scan over the query's own probe lists.  Each case checks that the stream path
ran, that the ids and score bits equal the oracle's and equal the exact path's (PYR_DEEP_REFINE=0), also with
every certificate forced to fail, up to k = 256 (the boundary's largest topK).
"""
import ctypes as C
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


class _env:
    def __init__(self, **kv):
        self.kv = {k: str(v) for k, v in kv.items()}

    def __enter__(self):
        self.old = {k: os.environ.get(k) for k in self.kv}
        os.environ.update(self.kv)

    def __exit__(self, *a):
        for k, v in self.old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def _sampled(lib, run):
    lib.pyr_profile_reset()
    lib.pyr_profile_enable(1)
    try:
        out = run()
    finally:
        lib.pyr_profile_enable(0)
    ms, calls, work = C.c_double(), C.c_int64(), C.c_int64()
    lib.pyr_profile_get(9, C.byref(ms), C.byref(calls), C.byref(work))
    return out, calls.value


def _bits(a, b):
    np.testing.assert_array_equal(a[2], b[2])
    np.testing.assert_array_equal(a[1], b[1])
    assert np.array_equal(a[0].view(np.uint32), b[0].view(np.uint32))


def _index(d, metric, n, nl, seed):
    from pyrope_amd import IvfFlatVectorIndex, generate_synthetic
    x = generate_synthetic(n, d, seed)
    idx = IvfFlatVectorIndex(d, metric, n_list=nl)
    idx.add_labels(np.arange(n, dtype=np.int64), x)
    idx.build()
    return idx, x


@pytest.mark.parametrize("metric", [0, 1, 2])
def test_ivf_large_k_matches_oracle(hiplib, oracle, metric):
    from pyrope_amd import SearchOptions, generate_synthetic
    idx, x = _index(128, metric, 12000, 24, 81)
    off, labels, live = idx.ivf_layout()
    rows = x[np.where(labels >= 0, labels, 0)]
    cents = idx.centroids_array()
    q = generate_synthetic(40, 128, 82)
    for k, P in [(61, 6), (100, 6), (124, 3), (200, 6), (252, 24), (256, 2)]:
        opts = SearchOptions(nprobe=P)
        got, calls = _sampled(hiplib, lambda: idx.search_batch(q, k, opts))
        assert calls >= 1, "k > 60 must take the stream scan"
        with _env(PYR_DEEP_REFINE=0):
            _bits(got, idx.search_batch(q, k, opts))
        s, l, c = got
        for i in range(0, len(q), 6):
            os_, ok = oracle.ivf_search(q[i], k, cents, rows, off, live, metric=metric, nprobe=P)
            assert int(c[i]) == len(os_), (k, i)
            np.testing.assert_array_equal(l[i][: len(ok)], labels[ok])
            assert np.array_equal(s[i][: len(os_)].view(np.uint32), os_.astype(np.float32).view(np.uint32))
    opts = SearchOptions(nprobe=6)
    ref = idx.search_batch(q, 150, opts)
    with _env(PYR_FILTER_CERR="1e15"):  # every certificate fails: the exact scan answers every query
        _bits(idx.search_batch(q, 150, opts), ref)
    idx.close()


def test_ivf_large_k_other_dim_and_past_range(hiplib, oracle):
    from pyrope_amd import SearchOptions, generate_synthetic
    idx, x = _index(96, 0, 8000, 16, 83)
    off, labels, live = idx.ivf_layout()
    rows = x[np.where(labels >= 0, labels, 0)]
    cents = idx.centroids_array()
    q = generate_synthetic(600, 96, 84)  # more than one item of 512 query slots per list
    opts = SearchOptions(nprobe=4)
    got, calls = _sampled(hiplib, lambda: idx.search_batch(q, 90, opts))
    assert calls >= 1
    with _env(PYR_DEEP_REFINE=0):
        _bits(got, idx.search_batch(q, 90, opts))
    for i in range(0, len(q), 97):
        os_, ok = oracle.ivf_search(q[i], 90, cents, rows, off, live, nprobe=4)
        np.testing.assert_array_equal(got[1][i][: len(ok)], labels[ok])
        assert np.array_equal(got[0][i][: len(os_)].view(np.uint32), os_.astype(np.float32).view(np.uint32))
    # k = 256, the boundary's largest topK: depth 512
    got, calls = _sampled(hiplib, lambda: idx.search_batch(q[:64], 256, opts))
    assert calls >= 1
    with _env(PYR_DEEP_REFINE=0):
        _bits(got, idx.search_batch(q[:64], 256, opts))
    for i in range(0, 64, 9):
        os_, ok = oracle.ivf_search(q[i], 256, cents, rows, off, live, nprobe=4)
        np.testing.assert_array_equal(got[1][i][: len(ok)], labels[ok])
        assert np.array_equal(got[0][i][: len(os_)].view(np.uint32), os_.astype(np.float32).view(np.uint32))
    idx.close()


@pytest.mark.parametrize("metric", [0, 1, 2])
def test_flat_large_k_matches_oracle(hiplib, oracle, metric):
    """FLAT L2 / IP / Cosine (BruteForceVectorIndex.cs:275-379, the *Unsafe forms; Cosine :354 on the raw rows)
    with k > 60 on the stream scan: the deep refine at V = 4 (Cosine: the unit store's scan, the exact Cosine in
    the refine, round 6), failures on the exact scan; equal to the oracle and to PYR_DEEP_REFINE=0"""
    from pyrope_amd import BruteForceVectorIndex, generate_synthetic
    n, d = 30000, 128
    x = generate_synthetic(n, d, 91)
    if metric == 2:  # signed rows with norms over a decade, and exact zero rows (cosine 0)
        x = (x - 0.5) * np.exp(np.linspace(0, 2.3, n, dtype=np.float32))[:, None]
        x[::997] = 0.0
        x = x.astype(np.float32)
    idx = BruteForceVectorIndex(d, metric)
    idx.add_labels(np.arange(n, dtype=np.int64), x)
    q = generate_synthetic(48, d, 92)
    if metric == 2:
        q = (q - 0.5).astype(np.float32)
    for k in [61, 150, 256]:
        got, calls = _sampled(hiplib, lambda: idx.search_batch(q, k))
        assert calls >= 1, "FLAT k > 60 must take the stream scan"
        with _env(PYR_DEEP_REFINE=0):
            _bits(got, idx.search_batch(q, k))
        for i in range(0, len(q), 7):
            os_, ok = oracle.bf_search(x, None, metric, q[i], k)
            np.testing.assert_array_equal(got[1][i], ok)
            assert np.array_equal(got[0][i].view(np.uint32), os_.astype(np.float32).view(np.uint32))
    with _env(PYR_FILTER_CERR="1e15"):
        ref = idx.search_batch(q, 100)
    with _env(PYR_DEEP_REFINE=0):
        _bits(idx.search_batch(q, 100), ref)
    idx.close()


@pytest.mark.parametrize("metric", [0, 2])
def test_ivf_large_k_with_buffer(hiplib, oracle, metric):
    """k > 60 with rows added after Build: the lists through the deep refine, the buffer's exact top k beside them,
    merged (merge_two_kernel, any k <= 256); equal to the oracle and to PYR_DEEP_REFINE=0"""
    from pyrope_amd import IvfFlatVectorIndex, SearchOptions, generate_synthetic
    d, n, nl, P = 128, 12000, 24, 6
    x = generate_synthetic(n, d, 95)
    idx = IvfFlatVectorIndex(d, metric, n_list=nl)
    idx.add_labels(np.arange(n, dtype=np.int64), x)
    idx.build()
    extra = generate_synthetic(300, d, 96)
    new_labels = np.concatenate([np.arange(n, n + 200), np.arange(0, 100)])
    idx.add_labels(new_labels, extra)
    off, labels, live = idx.ivf_layout()
    rows = x[np.where(labels >= 0, labels, 0)]
    cents = idx.centroids_array()
    slot_labels = new_labels.tolist()
    q = generate_synthetic(32, d, 97)
    for k in [80, 200]:
        opts = SearchOptions(nprobe=P)
        got, calls = _sampled(hiplib, lambda: idx.search_batch(q, k, opts))
        assert calls >= 1
        with _env(PYR_DEEP_REFINE=0):
            _bits(got, idx.search_batch(q, k, opts))
        for i in range(0, len(q), 5):
            os_, ok = oracle.ivf_search(q[i], k, cents, rows, off, live, buf=extra, metric=metric, nprobe=P)
            exp = np.array([slot_labels[kk - oracle.BUFKEY] if kk >= oracle.BUFKEY else labels[kk] for kk in ok],
                           np.int64)
            np.testing.assert_array_equal(got[1][i][: len(exp)], exp)
            assert np.array_equal(got[0][i][: len(os_)].view(np.uint32), os_.astype(np.float32).view(np.uint32))
    idx.close()


@pytest.mark.parametrize("metric", [0, 1, 2])
@pytest.mark.parametrize("max_scans", [1, 800, 3000])
def test_ivf_large_k_with_max_scans(hiplib, oracle, metric, max_scans):
    """k > 60 under a MaxScans budget (IvfFlatVectorIndex.cs:152-156, :202-212; round 6: the deep refine on the
    budgeted stream scan, its failures on the exact scan with the same budget over the lists alone); with and
    without rows in the buffer (which the budget reaches first), certificates as they fall and all forced to
    fail.  Equal to the oracle and to the exact path (PYR_DEEP_REFINE=0)."""
    from pyrope_amd import IvfFlatVectorIndex, SearchOptions, generate_synthetic
    d, n, nl, P = 128, 12000, 24, 6
    x = generate_synthetic(n, d, 101)
    idx = IvfFlatVectorIndex(d, metric, n_list=nl)
    idx.add_labels(np.arange(n, dtype=np.int64), x)
    idx.build()
    q = generate_synthetic(36, d, 102)
    off, labels, live = idx.ivf_layout()
    rows = x[np.where(labels >= 0, labels, 0)]
    cents = idx.centroids_array()
    opts = SearchOptions(nprobe=P, max_scans=max_scans)
    for k in [90, 200]:
        got, calls = _sampled(hiplib, lambda: idx.search_batch(q, k, opts))
        if max_scans > 1:
            assert calls >= 1, "k > 60 with a budget must take the stream scan"
        with _env(PYR_DEEP_REFINE=0):
            _bits(got, idx.search_batch(q, k, opts))
        with _env(PYR_FILTER_CERR="1e15"):
            _bits(got, idx.search_batch(q, k, opts))
        for i in range(0, len(q), 7):
            os_, ok = oracle.ivf_search(q[i], k, cents, rows, off, live, metric=metric, nprobe=P,
                                        max_scans=max_scans)
            assert int(got[2][i]) == len(os_)
            np.testing.assert_array_equal(got[1][i][: len(ok)], labels[ok])
            assert np.array_equal(got[0][i][: len(os_)].view(np.uint32), os_.astype(np.float32).view(np.uint32))
    # rows added after Build: the buffer takes its share of the budget first
    extra = generate_synthetic(150, d, 103)
    new_labels = np.concatenate([np.arange(n, n + 100), np.arange(0, 50)])
    idx.add_labels(new_labels, extra)
    off, labels, live = idx.ivf_layout()
    slot_labels = new_labels.tolist()
    got = idx.search_batch(q, 120, opts)
    with _env(PYR_DEEP_REFINE=0):
        _bits(got, idx.search_batch(q, 120, opts))
    with _env(PYR_FILTER_CERR="1e15"):
        _bits(got, idx.search_batch(q, 120, opts))
    for i in range(0, len(q), 7):
        os_, ok = oracle.ivf_search(q[i], 120, cents, rows, off, live, buf=extra, metric=metric, nprobe=P,
                                    max_scans=max_scans)
        exp = np.array([slot_labels[kk - oracle.BUFKEY] if kk >= oracle.BUFKEY else labels[kk] for kk in ok], np.int64)
        np.testing.assert_array_equal(got[1][i][: len(exp)], exp)
        assert np.array_equal(got[0][i][: len(os_)].view(np.uint32), os_.astype(np.float32).view(np.uint32))
    idx.close()
