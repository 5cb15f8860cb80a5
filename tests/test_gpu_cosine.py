"""Cosine FLAT search on the filter path (engine.cpp FlatIndex::search_cosine, filter.hip cos_rerank_kernel).

The candidates are the exact L2 top-K2 of the unit queries over the unit rows (an L2 FLAT index
over the same slots; on unit vectors the L2 order is the cosine order); their exact Cosine (BruteForceVectorIndex.cs:339-354: DotProductUnsafe
/ (|q| |x|), 0 when a norm is below 1e-6) is ranked and certified.  Results must be bit-identical to
the exact VALU scan (PYR_FILTER=0) and to the CPU oracle, through upserts with repeated ids, deletes,
MaxScans, zero-norm rows and queries, non-finite rows, ties and a snapshot / load round trip.
"""
import os

import numpy as np
import pytest

from test_gpu_filter import _env, _fallbacks, _same

pytestmark = pytest.mark.gpu

COS = 2


def _cos_index(dim, x, labels=None):
    from pyrope_amd import BruteForceVectorIndex
    idx = BruteForceVectorIndex(dim, COS)
    idx.add_labels(np.arange(len(x), dtype=np.int64) if labels is None else labels, x)
    return idx


def _check(idx, q, k, opts=None):
    got, nfb = _fallbacks(__import__("pyrope_amd")._lib.load(), lambda: idx.search_batch(q, k, opts))
    with _env(PYR_FILTER=0):
        ref = idx.search_batch(q, k, opts)
    _same(got, ref)
    return got, nfb


@pytest.mark.parametrize("k", [10, 20, 1])
@pytest.mark.parametrize("dim", [128, 64, 32])
def test_cosine_filter_equals_exact_and_oracle(hiplib, oracle, dim, k):
    from pyrope_amd import generate_synthetic
    x = generate_synthetic(20000, dim, 42)
    q = generate_synthetic(300, dim, 1337)
    idx = _cos_index(dim, x)
    got, nfb = _check(idx, q, k)
    for i in range(0, len(q), 37):
        os_, ok = oracle.bf_search(x, None, COS, q[i], k)
        np.testing.assert_array_equal(got[1][i], ok)
        assert np.array_equal(got[0][i].view(np.uint32), os_.view(np.uint32))
    print(f"\n[cos] dim={dim} k={k}: exact re-runs {nfb}/{len(q)}")
    # the certificate holds for almost every query (measured: at most 2 of 300 re-run)
    assert nfb < len(q) // 20


def test_cosine_signed_gaussian(hiplib, oracle):
    """Signed data: cosines over [-1, 1]; norms spread over two decades."""
    rng = np.random.default_rng(5)
    x = (rng.standard_normal((30000, 128)) * rng.uniform(0.01, 1.0, (30000, 1))).astype(np.float32)
    q = rng.standard_normal((200, 128)).astype(np.float32)
    idx = _cos_index(128, x)
    got, nfb = _check(idx, q, 10)
    for i in range(0, len(q), 23):
        os_, ok = oracle.bf_search(x, None, COS, q[i], 10)
        np.testing.assert_array_equal(got[1][i], ok)
        assert np.array_equal(got[0][i].view(np.uint32), os_.view(np.uint32))
    assert nfb < 20


def test_cosine_zero_norms_ties_nonfinite(hiplib, oracle):
    from pyrope_amd import generate_synthetic
    dim = 64
    x = generate_synthetic(5000, dim, 7) - 0.5
    x[10] = 0.0                      # zero norm: score 0 (VectorMath.cs:105 rule)
    x[11] = 1e-9                     # norm below 1e-6: score 0
    x[100:140] = x[7]                # 40 exact ties of one direction
    x[200:230] = x[8] * 3.0          # same direction, other norm
    q = generate_synthetic(64, dim, 9) - 0.5
    q[0] = 0.0                       # zero query: every score 0 -> lowest slots
    q[1] = x[7]
    q[2] = -x[8]
    idx = _cos_index(dim, x)
    got, nfb = _check(idx, q, 10)
    for i in range(8):
        os_, ok = oracle.bf_search(x, None, COS, q[i], 10)
        np.testing.assert_array_equal(got[1][i], ok)
        assert np.array_equal(got[0][i].view(np.uint32), os_.view(np.uint32))
    assert nfb >= 1  # the zero query re-runs exactly
    # a non-finite row: every certificate fails, results still equal the exact scan's
    x2 = x.copy()
    x2[300, 3] = np.inf
    idx2 = _cos_index(dim, x2)
    _check(idx2, q, 10)


def test_cosine_writes_deletes_maxscans_snapshot(hiplib, oracle, tmp_path):
    from pyrope_amd import BruteForceVectorIndex, SearchOptions, generate_synthetic
    dim = 128
    x = generate_synthetic(8000, dim, 3)
    q = generate_synthetic(100, dim, 4)
    idx = BruteForceVectorIndex(dim, COS)
    ids = [f"v{i}" for i in range(len(x))]
    idx.add_batch(ids, x)
    # one upsert batch with a repeated id (last write wins, slots out of order), new ids appended
    up = generate_synthetic(6, dim, 11)
    idx.upsert_batch(["v5", "new1", "v5", "v9", "new2", "new1"], up)
    for i in range(0, 8000, 97):
        idx.delete(f"v{i}")
    _check(idx, q, 10)
    _check(idx, q, 10, SearchOptions(max_scans=3000))
    # the host view: rows in slot order with deletions, compared with the oracle
    live_rows = np.stack([v for _, v in idx.scan()]).astype(np.float32)
    got = idx.search_batch(q, 10)
    for i in range(0, len(q), 19):
        os_, ok = oracle.bf_search(live_rows, None, COS, q[i], 10)
        assert np.array_equal(got[0][i].view(np.uint32), os_.view(np.uint32))
    path = os.path.join(str(tmp_path), "cos.idx")
    idx.snapshot(path)
    idx2 = BruteForceVectorIndex(dim, COS)
    idx2.load(path)
    got2 = _check(idx2, q, 10)[0]
    assert np.array_equal(got2[0].view(np.uint32), got[0].view(np.uint32))


# ---- IVF_FLAT Cosine (IvfFlatVectorIndex.cs:167, :357): the stream scan over unit residual tiles ----

def _list_scans(hiplib, fn):
    """stream sample-phase launches (PH_SAMPLE = 9) while fn() runs: only the IVF stream scan has one"""
    import ctypes as C
    hiplib.pyr_profile_reset()
    hiplib.pyr_profile_enable(1)
    try:
        fn()
    finally:
        hiplib.pyr_profile_enable(0)
    ms, calls, work = C.c_double(), C.c_int64(), C.c_int64()
    hiplib.pyr_profile_get(9, C.byref(ms), C.byref(calls), C.byref(work))
    return calls.value


def _ivf_cos(dim, x, nlist):
    from pyrope_amd import IvfFlatVectorIndex
    idx = IvfFlatVectorIndex(dim, COS, n_list=nlist)
    idx.add_labels(np.arange(len(x), dtype=np.int64), x)
    idx.build()
    return idx


def _ivf_oracle_check(idx, x, q, k, nprobe, oracle, step=1):
    from pyrope_amd import SearchOptions
    off, labels, live = idx.ivf_layout()
    rows = x[np.where(labels >= 0, labels, 0)]
    cents = idx.centroids_array()
    s, l, c = idx.search_batch(q, k, SearchOptions(nprobe=nprobe))
    for i in range(0, len(q), step):
        os_, ok = oracle.ivf_search(q[i], k, cents, rows, off, live, metric=COS, nprobe=nprobe)
        assert int(c[i]) == len(os_)
        np.testing.assert_array_equal(l[i][: len(ok)], labels[ok])
        assert np.array_equal(s[i][: len(os_)].view(np.uint32), os_.view(np.uint32))


@pytest.mark.parametrize("k", [10, 20])
@pytest.mark.parametrize("dim", [128, 64, 32])
def test_ivf_cosine_stream_equals_exact_and_oracle(hiplib, oracle, dim, k):
    from pyrope_amd import SearchOptions, generate_synthetic
    x = generate_synthetic(30000, dim, 42)
    q = generate_synthetic(200, dim, 1337)
    idx = _ivf_cos(dim, x, 64)
    got, nfb = _check(idx, q, k, SearchOptions(nprobe=8))
    print(f"\n[cos-ivf] dim={dim} k={k}: exact re-runs {nfb}/{len(q)}")
    assert _list_scans(hiplib, lambda: idx.search_batch(q, k, SearchOptions(nprobe=8))) > 0  # the stream path ran
    _ivf_oracle_check(idx, x, q, k, 8, oracle, step=13)
    assert nfb < len(q) // 10


def test_ivf_cosine_signed_zero_rows_deletes(hiplib, oracle):
    """Signed Gaussian clusters with norms over two decades, zero-norm rows (score 0), a zero query and
    deletes after Build (tombstones); every result equals the exact scan's and the oracle's."""
    from pyrope_amd import SearchOptions
    rng = np.random.default_rng(8)
    cent = rng.standard_normal((16, 128)).astype(np.float32)
    x = (cent[rng.integers(0, 16, 20000)] + 0.4 * rng.standard_normal((20000, 128))).astype(np.float32)
    x *= rng.uniform(0.01, 1.0, (20000, 1)).astype(np.float32)
    x[5] = 0.0
    x[77] = 1e-9
    q = (cent[rng.integers(0, 16, 120)] + 0.4 * rng.standard_normal((120, 128))).astype(np.float32)
    q[0] = 0.0
    q[1] = -q[2]
    idx = _ivf_cos(128, x, 32)
    opts = SearchOptions(nprobe=6)
    got, nfb = _check(idx, q, 10, opts)
    print(f"\n[cos-ivf] signed: exact re-runs {nfb}/{len(q)}")
    assert nfb >= 1 and nfb < len(q) // 4
    _ivf_oracle_check(idx, x, q, 10, 6, oracle, step=7)
    for i in range(0, 20000, 53):
        idx.delete(str(i))
    _check(idx, q, 10, opts)
    _ivf_oracle_check(idx, x, q, 10, 6, oracle, step=11)


