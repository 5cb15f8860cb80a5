"""The IVF list scan as the I1 bench runs it, plus the certificate's corner cases.

I1 (IVF_FLAT N=10M, nlist=1024) has lists of ~9.8k rows (max ~18k), so every list is split
into several row chunks (engine.cpp ivf_chunking, 5120 rows): per (query, probe, chunk)
partial slots and the chunk-aware merge (MergeIvf) are on the bench's path.  These tests
put lists longer than one chunk under the oracle -- with the default chunk on lists of
20k+ rows, and with PYR_IVF_CHUNK forcing many small chunks -- for L2 and IP, XCD-major
item mapping on and off, k = 10 and 40.  Reference: Vector/IvfFlatVectorIndex.cs:147-231
(list scan :200-218), VectorMath.cs:8-70.
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


def _same(a, b):
    (s1, l1, c1), (s2, l2, c2) = a, b
    np.testing.assert_array_equal(c1, c2)
    np.testing.assert_array_equal(l1, l2)
    assert np.array_equal(s1.view(np.uint32), s2.view(np.uint32))


def _fallbacks(hiplib, fn):
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


def _index(n, nl, metric):
    from pyrope_amd import IvfFlatVectorIndex, generate_synthetic
    key = (n, nl, metric)
    if key not in _CACHE:
        x = generate_synthetic(n, 128, 42)
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
@pytest.mark.parametrize("xcd", ["1", "0"])
def test_lists_longer_than_default_chunk(hiplib, oracle, metric, xcd):
    """200k rows in 8 lists: lists span several 5120-row chunks (the I1 shape; IP k-means on
    uniform data gives very uneven lists, 37 to 100k rows, which the chunking evens out)."""
    from pyrope_amd import SearchOptions, generate_synthetic
    idx, x = _index(200_000, 8, metric)
    off, _, _ = idx.ivf_layout()
    assert (np.diff(off) > 2 * 5120).sum() >= 3  # several lists of several chunks
    q = generate_synthetic(256, 128, 1337)
    opts = SearchOptions(nprobe=4)
    with _env(PYR_FILTER_XCD=xcd):
        got = idx.search_batch(q, 10, opts)
    with _env(PYR_FILTER=0):
        ref = idx.search_batch(q, 10, opts)
    _same(got, ref)
    _check_oracle(oracle, idx, x, q, got, 10, metric, 4, 32)


@pytest.mark.parametrize("metric", [0, 1])
@pytest.mark.parametrize("k", [10, 40])
@pytest.mark.parametrize("xcd", ["1", "0"])
@pytest.mark.parametrize("chunk", [64, 520])
def test_forced_small_chunks_nprobe32(hiplib, oracle, metric, k, xcd, chunk):
    """nprobe = 32 of 64 lists of ~1.6k rows, cut into PYR_IVF_CHUNK-row chunks (the chunk grows
    when nprobe x chunks would exceed the partial-slot budget)."""
    from pyrope_amd import SearchOptions, generate_synthetic
    idx, x = _index(100_000, 64, metric)
    q = generate_synthetic(300, 128, 1337)
    opts = SearchOptions(nprobe=32)
    with _env(PYR_IVF_CHUNK=chunk, PYR_FILTER_XCD=xcd):
        got = idx.search_batch(q, k, opts)
        with _env(PYR_FILTER=0):
            ref = idx.search_batch(q, k, opts)
    _same(got, ref)
    with _env(PYR_FILTER=0):  # and the exact scan with the default chunking
        ref2 = idx.search_batch(q, k, opts)
    _same(got, ref2)
    _check_oracle(oracle, idx, x, q, got, k, metric, 32, 60)


@pytest.mark.parametrize("chunk", [None, 256])
def test_caller_ranked_probes_with_failed_certificates(hiplib, chunk):
    """the exact re-run of queries whose certificate fails must scan THEIR
    probe lists when the caller hands the lists in (pyr_index_search_probed_device, the
    multi-GPU step).  Every certificate is forced to fail; results must equal the plain search."""
    import torch

    from pyrope_amd import SearchOptions, generate_synthetic
    idx, _ = _index(100_000, 64, 0)
    nq, npb = 500, 8
    qh = generate_synthetic(nq, 128, 99)
    opts = SearchOptions(nprobe=npb)
    env = {"PYR_FILTER_CERR": "1e15"}
    if chunk:
        env["PYR_IVF_CHUNK"] = str(chunk)
    with _env(**env):
        ref = idx.search_batch(qh, 10, opts)
        q = torch.from_numpy(qh).cuda()
        probes = torch.empty((nq, npb), dtype=torch.int32, device="cuda")
        stream = torch.cuda.current_stream().cuda_stream
        assert idx.probe_device(q.data_ptr(), nq, probes.data_ptr(), stream, opts) == npb
        probes = probes.flip(1).contiguous()  # any column order names the same lists
        s = torch.empty((nq, 10), dtype=torch.float32, device="cuda")
        lab = torch.empty((nq, 10), dtype=torch.int64, device="cuda")
        (_, nfb) = _fallbacks(hiplib, lambda: (idx.search_device(q.data_ptr(), nq, 10, s.data_ptr(), lab.data_ptr(),
                                                                  0, stream, opts, d_probes=probes.data_ptr(),
                                                                  nprobe=npb), torch.cuda.synchronize()))
    assert nfb >= nq  # every query re-run (filter tier, then exact)
    np.testing.assert_array_equal(lab.cpu().numpy(), ref[1])
    assert np.array_equal(s.cpu().numpy().view(np.uint32), ref[0].view(np.uint32))


def _clustered(n, nclu, d, seed, outliers):
    rng = np.random.default_rng(seed)
    centers = rng.standard_normal((nclu, d)).astype(np.float32) * 4
    lab = rng.integers(0, nclu, n)
    x = (centers[lab] + rng.standard_normal((n, d)).astype(np.float32)).astype(np.float32)
    far = rng.choice(n, outliers, replace=False)
    x[far] *= 300.0  # a few rows with ~300x the typical norm
    q = (centers[rng.integers(0, nclu, 400)] + rng.standard_normal((400, d)).astype(np.float32)).astype(np.float32)
    return x, q


@pytest.mark.parametrize("metric", [0, 1])
def test_per_list_certificate_on_skewed_data(hiplib, metric):
    """Gaussian clusters with a few large-norm outliers (k-means puts them in hub
    lists that nearly every query probes).  The certificate bounds row norms by the probed lists'
    maxima and, for L2, by |q| + sqrt(-s_k) (rows beyond cannot reach the k-th score), so the
    outliers cost nothing; the index-wide bound alone (PYR_CERT_GLOBAL=1) fails every query.
    Results are identical either way (failures re-run exactly)."""
    from pyrope_amd import IvfFlatVectorIndex, SearchOptions
    x, q = _clustered(60_000, 64, 128, 3, 6)
    idx = IvfFlatVectorIndex(128, metric, n_list=64)
    idx.add_labels(np.arange(len(x), dtype=np.int64), x)
    idx.build()
    opts = SearchOptions(nprobe=8)
    with _env(PYR_FILTER=0):
        ref = idx.search_batch(q, 10, opts)
    # the bf16x3 filter's certificate (|q| |x|-relative error): per-list maxima + triangle bound
    # against the index-wide maximum alone
    with _env(PYR_FILTER_PREC=1, PYR_FILTER_TIER=0):
        got, nfb_list = _fallbacks(hiplib, lambda: idx.search_batch(q, 10, opts))
        with _env(PYR_CERT_GLOBAL=1):
            got_g, nfb_global = _fallbacks(hiplib, lambda: idx.search_batch(q, 10, opts))
    _same(got, ref)
    _same(got_g, ref)
    # the default path (stream16.hip over fp16 residual tiles): candidates carry per-row upper bounds
    # (stream_ub_terms), so an outlier inflates only its own row's bound, not its list's; the sample
    # rank adapts to these short, mostly-sampled lists (sselect_kernel).  Round 2 re-ran 254 / 296 of
    # the 400 queries here; now at most 1 % may fail.
    got16, nfb16 = _fallbacks(hiplib, lambda: idx.search_batch(q, 10, opts))
    _same(got16, ref)
    print(f"\n[cert] metric={metric}: bf16x3 exact re-runs per-list bound {nfb_list}/{len(q)}, "
          f"index-wide bound {nfb_global}/{len(q)}; fp16 stream re-runs {nfb16}/{len(q)}")
    assert nfb_list <= nfb_global
    if metric == 0:
        assert nfb_list < len(q) // 10
    assert nfb16 <= len(q) // 100


@pytest.mark.parametrize("metric", [0, 1])
@pytest.mark.parametrize("wide,prio,waves,k", [("1", "2", "4", 10), ("1", "0", "4", 10), ("1", "1", "4", 10),
                                               ("0", "0", "4", 10), ("1", "2", "16", 10), ("1", "2", "4", 20),
                                               ("0", "0", "4", 20)])
def test_both_list_scan_kernels(hiplib, oracle, metric, wide, prio, waves, k):
    """The K1 = 16 / 32 list scan (k = 10 / 20) runs on the 8-wave x 16-query kernel (mfma_filter16w:
    top-K1 spread over a query's 4 lanes, 16x16x32 MFMA) by default and on the 4-wave x 32-query kernel with
    PYR_F16_WIDE=0; PYR_FILTER_WAVES=16 runs 256-query items on 16-wave blocks; the priority
    modes only reorder the waves.  Every setting must give the
    exact scan's answers bit for bit, on multi-chunk lists (small forced chunks) and a full
    128-query group per item."""
    from pyrope_amd import SearchOptions, generate_synthetic
    idx, x = _index(100_000, 64, metric)
    q = generate_synthetic(700, 128, 4242)
    opts = SearchOptions(nprobe=16)
    with _env(PYR_F16_WIDE=wide, PYR_F16_PRIO=prio, PYR_FILTER_WAVES=waves, PYR_IVF_CHUNK=520):
        got = idx.search_batch(q, k, opts)
    with _env(PYR_FILTER=0):
        ref = idx.search_batch(q, k, opts)
    _same(got, ref)
    _check_oracle(oracle, idx, x, q, got, k, metric, 16, 100)


@pytest.mark.parametrize("metric", [0, 1])
def test_coarse_ranking_through_flat_filter(hiplib, metric):
    """PYR_COARSE_FILTER=1 (read when the centroids are set): the coarse step runs as a FLAT filter
    search over the centroids (fp16 tiles, K1 = 64, exact safe-form refine = ComputeScore,
    IvfFlatVectorIndex.cs:186-198).  The probes, hence the answers, equal the dense exact ranking."""
    from pyrope_amd import IvfFlatVectorIndex, SearchOptions, generate_synthetic
    x = generate_synthetic(40_000, 128, 42)
    q = generate_synthetic(500, 128, 1337)
    opts = SearchOptions(nprobe=32)
    with _env(PYR_COARSE_FILTER=1):
        idx = IvfFlatVectorIndex(128, metric, n_list=256)
        idx.add_labels(np.arange(len(x), dtype=np.int64), x)
        idx.build()
        got = idx.search_batch(q, 10, opts)
    with _env(PYR_FILTER=0):  # exact list scan and the dense exact coarse ranking
        ref = idx.search_batch(q, 10, opts)
    _same(got, ref)
