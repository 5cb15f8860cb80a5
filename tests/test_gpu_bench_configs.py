"""The coarse / probe configurations the benches run, under the oracle.

I1 ranks nlist = 1024 centroids with nprobe = 32, M8 8192 with nprobe = 32 (and 64 here), P1 4096
with nprobe = 64 on d = 768 / M = 96 codes.  The coarse selection kernel is instantiated by list count
and nprobe (coarse.hip coarse_select_reg_kernel<16> at 1024 centroids, <32> at nprobe = 32 and <64>
at nprobe = 64 over 4096 / 8192), so these sizes reach code the small-nlist tests never run.  N stays small (a few to a few tens of rows
per list), and the quantizers are supplied (pyr_index_set_centroids / set_codebooks: sampled rows),
so every case takes seconds.  Reference: Vector/IvfFlatVectorIndex.cs:186-198 (ranking) and
:200-218 (list scan), Vector/IvfPqVectorIndex.cs:141-198, ProductQuantizer.cs:98-120.
"""
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


_CACHE = {}


def _ivf(nlist, per_list, metric, dim=128):
    from pyrope_amd import IvfFlatVectorIndex, generate_synthetic
    key = (nlist, per_list, metric, dim)
    if key not in _CACHE:
        n = nlist * per_list
        x = generate_synthetic(n, dim, 42)
        rng = np.random.default_rng(nlist)
        cents = x[rng.choice(n, nlist, replace=False)].copy()
        idx = IvfFlatVectorIndex(dim, metric, n_list=nlist)
        idx.set_centroids(cents)
        idx.add_labels(np.arange(n, dtype=np.int64), x)
        idx.build()
        _CACHE[key] = (idx, x)
    return _CACHE[key]


@pytest.mark.parametrize("metric", [0, 1])
@pytest.mark.parametrize("nlist,nprobe,per_list", [(1024, 32, 40), (4096, 64, 12), (8192, 32, 12), (8192, 64, 12)])
def test_ivf_flat_bench_coarse_configs(hiplib, oracle, metric, nlist, nprobe, per_list):
    """I1 / M8-shaped coarse ranking + list scan vs the exact VALU path and the oracle."""
    from pyrope_amd import SearchOptions, generate_synthetic
    idx, x = _ivf(nlist, per_list, metric)
    q = generate_synthetic(600, 128, 1337)
    opts = SearchOptions(nprobe=nprobe)
    got = idx.search_batch(q, 10, opts)
    with _env(PYR_FILTER=0):
        ref = idx.search_batch(q, 10, opts)
    _same(got, ref)
    off, labels, live = idx.ivf_layout()
    rows = x[np.where(labels >= 0, labels, 0)]
    cents = idx.centroids_array()
    for i in range(0, len(q), 47):
        os_, ok = oracle.ivf_search(q[i], 10, cents, rows, off, live, metric=metric, nprobe=nprobe)
        np.testing.assert_array_equal(got[1][i][: len(ok)], labels[ok])
        assert np.array_equal(got[0][i][: len(ok)].view(np.uint32), os_.view(np.uint32))


@pytest.mark.parametrize("nlist", [1024, 8192])
def test_probe_lists_equal_oracle_ranking(hiplib, oracle, nlist):
    """pyr_index_probe_device (the multi-GPU step's coarse split) at the bench list counts: the
    probe SET of every query equals the oracle's top-nprobe ranking (ComputeScore, ties -> lower
    centroid index)."""
    import torch

    from pyrope_amd import SearchOptions, generate_synthetic
    idx, _ = _ivf(nlist, 12 if nlist > 1024 else 40, 0)
    nq, npb = 200, 32
    qh = generate_synthetic(nq, 128, 7)
    q = torch.from_numpy(qh).cuda()
    pr = torch.empty((nq, npb), dtype=torch.int32, device="cuda")
    assert idx.probe_device(q.data_ptr(), nq, pr.data_ptr(), 0, SearchOptions(nprobe=npb)) == npb
    torch.cuda.synchronize()
    got = pr.cpu().numpy()
    cents = idx.centroids_array()
    for i in range(0, nq, 19):
        exp = np.asarray(oracle.ivf_probe(qh[i], cents, npb, metric=0))
        assert sorted(got[i].tolist()) == sorted(exp.tolist())


@pytest.mark.parametrize("nlist,nprobe", [(256, 64), (4096, 64)])
def test_ivf_pq_p1_geometry(hiplib, oracle, nlist, nprobe):
    """P1 geometry: d = 768, M = 96 (8-dim subspaces), K = 256, nprobe = 64, with supplied quantizers
    (the P1 bulk path) -- LUT, ADC and ranking bit-identical to the oracle."""
    from pyrope_amd import IvfPqVectorIndex, SearchOptions, generate_synthetic
    d, m, ksub = 768, 96, 256
    n = nlist * 6
    x = generate_synthetic(n, d, 42)
    rng = np.random.default_rng(5)
    cents = x[rng.choice(n, nlist, replace=False)].copy()
    sub = x[rng.choice(n, ksub, replace=False)].reshape(ksub, m, d // m)
    cb = np.ascontiguousarray(sub.transpose(1, 0, 2))  # [M][ksub][d / M]
    idx = IvfPqVectorIndex(d, 0, m=m, k=ksub, n_list=nlist)
    idx.set_centroids(cents)
    idx.set_codebooks(cb)
    idx.add_labels(np.arange(n, dtype=np.int64), x)
    idx.build()
    gcb, codes, off, labels, live = idx.pq_state()
    assert np.array_equal(gcb.view(np.uint32), cb.view(np.uint32))
    q = generate_synthetic(64, d, 1337)
    s, l, c = idx.search_batch(q, 10, SearchOptions(nprobe=nprobe))
    gc = idx.centroids_array()
    for i in range(0, len(q), 9):
        os_, ok = oracle.ivfpq_search(q[i], 10, gc, codes, off, gcb, live, metric=0, nprobe=nprobe)
        assert int(c[i]) == len(os_)
        np.testing.assert_array_equal(l[i][: len(ok)], labels[ok])
        assert np.array_equal(s[i][: len(os_)].view(np.uint32), os_.view(np.uint32))


def _probe_sets(idx, qh, npb, **env):
    import torch

    from pyrope_amd import SearchOptions
    q = torch.from_numpy(qh).cuda()
    pr = torch.empty((len(qh), npb), dtype=torch.int32, device="cuda")
    with _env(**env):
        assert idx.probe_device(q.data_ptr(), len(qh), pr.data_ptr(), 0, SearchOptions(nprobe=npb)) == npb
    torch.cuda.synchronize()
    return pr.cpu().numpy()


@pytest.mark.parametrize("metric", [0, 1])
@pytest.mark.parametrize("nlist,npb", [(1024, 32), (8192, 32), (8192, 64), (300, 16), (40, 40)])
def test_mfma_coarse_ranking_equals_dense_exact(hiplib, metric, nlist, npb):
    """The matrix-core coarse ranking (fp32 MFMA approximate scores, the exact ComputeScore of every
    centroid within the error band of the nprobe-th; coarse.hip launch_coarse_mfma) gives the dense
    exact ranking's probe lists, in order, for every query -- also when every query is forced through the in-kernel fallback
    (PYR_COARSE_CERR=1e15), and on clustered queries whose centroid scores are tightly packed."""
    from pyrope_amd import generate_synthetic
    idx, x = _ivf(nlist, 12 if nlist > 1024 else 40, metric)
    rng = np.random.default_rng(3)
    qh = np.concatenate([generate_synthetic(300, 128, 11),
                         (x[rng.choice(len(x), 200)] + 1e-3 * rng.standard_normal((200, 128))).astype(np.float32)])
    ref = _probe_sets(idx, qh, npb, PYR_COARSE_MFMA=0)
    np.testing.assert_array_equal(_probe_sets(idx, qh, npb), ref)
    np.testing.assert_array_equal(_probe_sets(idx, qh, npb, PYR_COARSE_CERR="1e15"), ref)


def test_mfma_coarse_ranking_ties_and_duplicate_centroids(hiplib):
    """Duplicated centroids give exactly tied scores: the lower centroid index ranks first
    (IvfFlatVectorIndex.cs:186-198 sorted with the index as the tie rule)."""
    from pyrope_amd import IvfFlatVectorIndex, generate_synthetic
    base = generate_synthetic(128, 128, 5)
    cents = np.repeat(base, 4, axis=0)  # every centroid four times
    x = generate_synthetic(4096, 128, 6)
    idx = IvfFlatVectorIndex(128, 0, n_list=len(cents))
    idx.set_centroids(cents)
    idx.add_labels(np.arange(len(x), dtype=np.int64), x)
    idx.build()
    qh = generate_synthetic(200, 128, 7)
    ref = _probe_sets(idx, qh, 24, PYR_COARSE_MFMA=0)
    got = _probe_sets(idx, qh, 24)
    np.testing.assert_array_equal(got, ref)
    assert (np.diff(got[:, :4], axis=1) == 1).all()  # the four copies of the best centroid, in index order


@pytest.mark.parametrize("metric", [0, 1])
@pytest.mark.parametrize("dim", [32, 64, 256])
def test_bf16_split_coarse_ranking_wide_magnitudes(hiplib, metric, dim):
    """The bf16 hi / lo split approximate scores (coarse.hip coarse_approx_bf3_kernel, the default when the
    dimension is a multiple of 16) against the dense exact ranking and the fp32 MFMA kernel
    (PYR_COARSE_APPROX=1): signed data whose dimensions span six decades of scale (the split's lo parts
    span as many), centroids drawn near the queries (tightly packed scores), nlist not a multiple of 32."""
    from pyrope_amd import IvfFlatVectorIndex
    rng = np.random.default_rng(dim + metric)
    scale = (10.0 ** rng.uniform(-3, 3, dim)).astype(np.float32)
    nlist = 333
    x = (rng.standard_normal((nlist * 8, dim)) * scale).astype(np.float32)
    cents = x[rng.choice(len(x), nlist, replace=False)].copy()
    idx = IvfFlatVectorIndex(dim, metric, n_list=nlist)
    idx.set_centroids(cents)
    idx.add_labels(np.arange(len(x), dtype=np.int64), x)
    idx.build()
    qh = np.concatenate([(rng.standard_normal((150, dim)) * scale).astype(np.float32),
                         (cents[rng.choice(nlist, 150)] * (1 + 1e-4 * rng.standard_normal((150, dim)))).astype(np.float32)])
    ref = _probe_sets(idx, qh, 16, PYR_COARSE_MFMA=0)
    np.testing.assert_array_equal(_probe_sets(idx, qh, 16), ref)
    np.testing.assert_array_equal(_probe_sets(idx, qh, 16, PYR_COARSE_APPROX=1), ref)


def test_work_lists_sixteen_entries_per_thread(hiplib):
    """A batch of >= 2M (query, probe) entries takes the 16-entries-per-thread work-list kernels
    (kernels.hip ivf_ept; a list-sharded rank's N x batch): 65,536 queries x nprobe 32 on a small index, against
    the exact VALU path."""
    from pyrope_amd import SearchOptions, generate_synthetic
    idx, _ = _ivf(256, 40, 0)
    q = generate_synthetic(65_536, 128, 2024)
    opts = SearchOptions(nprobe=32)
    got = idx.search_batch(q, 10, opts)
    with _env(PYR_FILTER=0):
        ref = idx.search_batch(q, 10, opts)
    _same(got, ref)
