"""The rows-as-A list scan (filter16r.hip, default for the fp16 IVF filter at K1 = 16 / 32) and the
configurations the bench runs.

mfma_filter16r serves up to 512 queries per (list, row chunk) item on 16 waves, keeps candidates in
per-lane top-8 lists and writes KEY_FLOOR placeholders where a lane may have dropped rows; its
answers must equal the exact scan's (PYR_FILTER=0) and the round-2 kernel's (PYR_F16_RK=0) bit for
bit, and the oracle's.  Cases: L2 / IP, k = 10 / 20 (K1 16 / 32), one- and two-term fp16 queries,
XCD mapping on / off, lists probed by more than 512 queries (several balanced items per chunk),
forced small chunks, 4-deep lane lists (PYR_RK_L=4: floors reach the top-K1 often), clustered data,
and the bench's coarse shapes nlist = 1024 / 8192 at nprobe = 32 / 64 (coarse_select_reg_kernel
<16>, <32>, <64>).  Reference: Vector/IvfFlatVectorIndex.cs:147-231, VectorMath.cs:8-70.
"""
import ctypes as C
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _rk_on(monkeypatch):
    monkeypatch.setenv("PYR_F16_RK", "1")  # the kernel under test (opt-in while it is tuned)


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


def _same(a, b):
    (s1, l1, c1), (s2, l2, c2) = a, b
    np.testing.assert_array_equal(c1, c2)
    np.testing.assert_array_equal(l1, l2)
    assert np.array_equal(s1.view(np.uint32), s2.view(np.uint32))


def _reruns(hiplib, fn):
    hiplib.pyr_profile_reset()
    hiplib.pyr_profile_enable(1)
    try:
        out = fn()
    finally:
        hiplib.pyr_profile_enable(0)
    ms, calls, work = C.c_double(), C.c_int64(), C.c_int64()
    hiplib.pyr_profile_get(8, C.byref(ms), C.byref(calls), C.byref(work))
    return out, work.value


_CACHE = {}


def _index(n, nl, metric, seed=42):
    from pyrope_amd import IvfFlatVectorIndex, generate_synthetic
    key = (n, nl, metric, seed)
    if key not in _CACHE:
        x = generate_synthetic(n, 128, seed)
        idx = IvfFlatVectorIndex(128, metric, n_list=nl)
        idx.add_labels(np.arange(n, dtype=np.int64), x)
        idx.build()
        _CACHE[key] = (idx, x)
    return _CACHE[key]


def _check_oracle(oracle, idx, x, q, got, k, metric, nprobe, step):
    off, labels, live = idx.ivf_layout()
    rows = x[np.where(labels >= 0, labels, 0)]
    cents = idx.centroids_array()
    for i in range(0, len(q), step):
        os_, ok = oracle.ivf_search(q[i], k, cents, rows, off, live, metric=metric, nprobe=nprobe)
        np.testing.assert_array_equal(got[1][i][: len(ok)], labels[ok])
        assert np.array_equal(got[0][i][: len(ok)].view(np.uint32), os_.view(np.uint32))


@pytest.mark.parametrize("metric", [0, 1])
@pytest.mark.parametrize("k", [10, 20])
@pytest.mark.parametrize("prec", ["2", "3"])
@pytest.mark.parametrize("xcd", ["1", "0"])
def test_rk_equals_exact_and_round2_kernel(hiplib, oracle, metric, k, prec, xcd):
    """2,000 queries x nprobe 16 over 64 lists: ~500 queries per list, so lists get one or two
    balanced items per chunk; forced 520-row chunks put several chunks per list."""
    from pyrope_amd import SearchOptions, generate_synthetic
    idx, x = _index(100_000, 64, metric)
    q = generate_synthetic(2000, 128, 4242)
    opts = SearchOptions(nprobe=16)
    with _env(PYR_FILTER_PREC=prec, PYR_FILTER_XCD=xcd, PYR_IVF_CHUNK=520):
        got = idx.search_batch(q, k, opts)
        with _env(PYR_F16_RK=0):
            old = idx.search_batch(q, k, opts)
    with _env(PYR_FILTER=0):
        ref = idx.search_batch(q, k, opts)
    _same(got, ref)
    _same(old, ref)
    _check_oracle(oracle, idx, x, q, got, k, metric, 16, 250)


@pytest.mark.parametrize("metric", [0, 1])
def test_rk_many_queries_per_list(hiplib, metric):
    """6,000 queries x nprobe 8 of 16 lists: ~3,000 queries per list -> 6 balanced 512-query items per
    chunk (the per-list query split, kernels.hip ivf_items_kernel)."""
    from pyrope_amd import SearchOptions, generate_synthetic
    idx, _ = _index(60_000, 16, metric)
    q = generate_synthetic(6000, 128, 77)
    opts = SearchOptions(nprobe=8)
    got = idx.search_batch(q, 10, opts)
    with _env(PYR_FILTER=0):
        ref = idx.search_batch(q, 10, opts)
    _same(got, ref)


def _clustered(n, nclu, d, seed, nq):
    rng = np.random.default_rng(seed)
    centers = rng.standard_normal((nclu, d)).astype(np.float32) * 4
    lab = rng.integers(0, nclu, n)
    x = (centers[lab] + rng.standard_normal((n, d)).astype(np.float32)).astype(np.float32)
    q = (centers[rng.integers(0, nclu, nq)] + rng.standard_normal((nq, d)).astype(np.float32)).astype(np.float32)
    return x, q


@pytest.mark.parametrize("metric", [0, 1])
@pytest.mark.parametrize("lanes", ["8", "4"])
def test_rk_floors_on_clustered_data(hiplib, metric, lanes):
    """Gaussian clusters: a query's best rows sit in one list, so a lane can see more of them than
    its list holds.  With 4-deep lists (PYR_RK_L=4) floors reach the merged top-K1 for many queries:
    the KEY_FLOOR placeholders must keep the certificate sound (failures re-run, answers exact)."""
    from pyrope_amd import IvfFlatVectorIndex, SearchOptions
    x, q = _clustered(50_000, 32, 128, 5, 600)
    idx = IvfFlatVectorIndex(128, metric, n_list=32)
    idx.add_labels(np.arange(len(x), dtype=np.int64), x)
    idx.build()
    opts = SearchOptions(nprobe=4)
    with _env(PYR_FILTER=0):
        ref = idx.search_batch(q, 10, opts)
    with _env(PYR_RK_L=lanes):
        got, nre = _reruns(hiplib, lambda: idx.search_batch(q, 10, opts))
    _same(got, ref)
    print(f"\n[rk floors] metric={metric} lane depth {lanes}: re-runs {nre}/{len(q)}")


@pytest.mark.parametrize("metric", [0, 1])
@pytest.mark.parametrize("nl,npb,n", [(1024, 32, 200_000), (8192, 32, 400_000), (8192, 64, 400_000)])
def test_bench_coarse_shapes(hiplib, oracle, metric, nl, npb, n):
    """The coarse selection at the bench's shapes (I1: nlist 1024 / nprobe 32; M8: 8192 / 32; and
    8192 / 64), small lists so that the oracle finishes in seconds."""
    from pyrope_amd import SearchOptions, generate_synthetic
    idx, x = _index(n, nl, metric, seed=11)
    q = generate_synthetic(1000, 128, 1337)
    opts = SearchOptions(nprobe=npb)
    got = idx.search_batch(q, 10, opts)
    with _env(PYR_FILTER=0):
        ref = idx.search_batch(q, 10, opts)
    _same(got, ref)
    _check_oracle(oracle, idx, x, q, got, 10, metric, npb, 100)
