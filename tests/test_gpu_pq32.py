"""The matrix-core IVF_PQ scan (pq32.hip) against the LUT scan and the oracle.

IvfPqVectorIndex.Search (IvfPqVectorIndex.cs:118-212) ranks by the fp32 ADC sum; pq32 reaches it through
an fp16 decode-and-MFMA filter, the reference's own table sum for the best candidates, and a certificate,
with the LUT scan re-running what fails.  Every test asserts that pq32 actually ran (its sample phase
shows in the profiler) and compares ids and score bits.
"""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

PH_FALLBACK, PH_SAMPLE = 8, 9


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


def _profiled(hiplib, fn):
    """fn() with the phase profiler on; returns (result, {phase: (calls, work)})."""
    hiplib.pyr_profile_reset()
    hiplib.pyr_profile_enable(1)
    try:
        out = fn()
    finally:
        hiplib.pyr_profile_enable(0)
    ph = {}
    for p in (PH_FALLBACK, PH_SAMPLE):
        ms, calls, work = C.c_double(), C.c_int64(), C.c_int64()
        hiplib.pyr_profile_get(p, C.byref(ms), C.byref(calls), C.byref(work))
        ph[p] = (calls.value, work.value)
    return out, ph


def _same(a, b):
    np.testing.assert_array_equal(a[1], b[1])
    assert np.array_equal(np.asarray(a[0]).view(np.uint32), np.asarray(b[0]).view(np.uint32))


def _build(dim, m, n, nlist, ksub=256, seed=42):
    from pyrope_amd import IvfPqVectorIndex, generate_synthetic
    x = generate_synthetic(n, dim, seed)
    idx = IvfPqVectorIndex(dim, 0, m=m, k=ksub, n_list=nlist)
    idx.add_labels(np.arange(n, dtype=np.int64), x)
    idx.build()
    return idx, x


@pytest.mark.parametrize("slice_q", [None, 7])
def test_pq32_caller_probes_with_failed_certificates(hiplib, slice_q):
    """with caller-ranked probe lists (pyr_index_search_probed_device), every query
    slice must scan its own rows of the lists, and the LUT re-run of failed certificates must scan the
    caller's lists too (not the coarse ranking's).  The lists here are random, so either slip changes
    the answers.  Each case runs as it falls and with every certificate forced to fail."""
    import torch

    from pyrope_amd import SearchOptions, generate_synthetic
    d, m, nl, P, nq, k = 768, 96, 12, 4, 40, 10
    idx, _ = _build(d, m, 3000, nl)
    rng = np.random.default_rng(3)
    probes = np.stack([rng.choice(nl, P, replace=False) for _ in range(nq)]).astype(np.int32)
    qh = generate_synthetic(nq, d, 99)
    q = torch.from_numpy(qh).cuda()
    pr = torch.from_numpy(probes).cuda()
    opts = SearchOptions(nprobe=P)

    def run():
        s = torch.empty((nq, k), dtype=torch.float32, device="cuda")
        lab = torch.empty((nq, k), dtype=torch.int64, device="cuda")
        idx.search_device(q.data_ptr(), nq, k, s.data_ptr(), lab.data_ptr(), 0, 0, opts, d_probes=pr.data_ptr(),
                          nprobe=P)
        torch.cuda.synchronize()
        return s.cpu().numpy(), lab.cpu().numpy()

    base = {"PYR_SLICE_QUERIES": slice_q} if slice_q else {}
    with _env(PYR_PQ_MFMA=0):
        ref = run()
    for force in (False, True):
        env = dict(base, PYR_FILTER_CERR="1e15") if force else base
        with _env(**env):
            got, ph = _profiled(hiplib, run)
        assert ph[PH_SAMPLE][0] > 0  # the pq32 path ran
        if force:
            assert ph[PH_FALLBACK][1] == nq  # every query re-ran on the LUT scan
        _same(got, ref)
    # and the lists really differ from the coarse ranking's (the test would not see a slip otherwise)
    plain = idx.search_batch(qh, k, opts)
    assert not np.array_equal(plain[1], ref[1])


# (dim, m): dsub 4 / 8 / 16 / 32 on both tile loops (KS = dim / 16 <= 8: decoded rows resident, 16 query
# groups per item; KS > 8: k-outer with 4 / 3 / 2 groups), the registry default (d=128, m=4,
# VectorIndexRegistry.cs:96-101), the reference's test geometry (d=128, m=16, IvfPqVectorIndexTests.cs:41-67)
# and P1's (d=768, m=96)
_GEOMS = [(128, 4), (128, 8), (128, 16), (128, 32), (96, 12), (64, 16), (256, 16), (512, 16), (384, 96),
          (768, 24), (768, 96), (1024, 64)]


@pytest.mark.parametrize("dim,m", _GEOMS)
def test_pq32_geometries_equal_lut_and_oracle(hiplib, oracle, dim, m):
    from pyrope_amd import SearchOptions, generate_synthetic
    n = 6000 if dim <= 256 else 3000
    idx, x = _build(dim, m, n, 12)
    q = generate_synthetic(1500, dim, 99)  # ~625 queries per probed list: several items per list chunk
    opts = SearchOptions(nprobe=5)
    for k in (1, 10, 60):
        got, ph = _profiled(hiplib, lambda: idx.search_batch(q, k, opts))
        assert ph[PH_SAMPLE][0] > 0, "the pq32 path did not run"
        with _env(PYR_PQ_MFMA=0):
            ref = idx.search_batch(q, k, opts)
        np.testing.assert_array_equal(got[2], ref[2])
        _same(got, ref)
    cb, codes, off, labels, live = idx.pq_state()
    cents = idx.centroids_array()
    for i in range(0, len(q), 151):
        os_, ok = oracle.ivfpq_search(q[i], 10, cents, codes, off, cb, live, metric=0, nprobe=5)
        s, lab, c = idx.search_batch(q[i:i + 1], 10, opts)
        np.testing.assert_array_equal(lab[0][: len(ok)], labels[ok])
        assert np.array_equal(s[0][: len(os_)].view(np.uint32), os_.view(np.uint32))


@pytest.mark.parametrize("dim,m", [(128, 4), (768, 96)])
def test_pq32_small_chunks_and_forced_failures(hiplib, dim, m):
    """Lists cut into 64-row chunks (many items per list, XCD queues with several items each) and every
    certificate forced to fail (all queries re-run on the LUT scan): still the LUT scan's answers."""
    from pyrope_amd import SearchOptions, generate_synthetic
    idx, _ = _build(dim, m, 4000, 12)
    q = generate_synthetic(300, dim, 7)
    opts = SearchOptions(nprobe=4)
    with _env(PYR_PQ_MFMA=0):
        ref = idx.search_batch(q, 10, opts)
    with _env(PYR_STREAM_CHUNK=64):
        got, ph = _profiled(hiplib, lambda: idx.search_batch(q, 10, opts))
    assert ph[PH_SAMPLE][0] > 0
    _same(got, ref)
    with _env(PYR_FILTER_CERR="1e15"):
        got, ph = _profiled(hiplib, lambda: idx.search_batch(q, 10, opts))
    assert ph[PH_FALLBACK][1] == len(q)
    _same(got, ref)


@pytest.mark.parametrize("dim,m", [(128, 4), (768, 96)])
def test_pq32_with_buffer_rows(hiplib, oracle, dim, m):
    """A non-empty buffer (rows added after Build, IvfPqVectorIndex.cs:130-136): the lists run on pq32 and the
    buffer exactly beside them, merged (a list entry first on equal scores).  New ids, ids that shadow their
    list entries (:134, :170) and a deleted buffer row; as the certificates fall and with all forced to fail
    (the LUT re-run then takes the lists only).  Equal to the LUT path and to the oracle."""
    from pyrope_amd import SearchOptions, generate_synthetic
    n = 4000
    idx, x = _build(dim, m, n, 12)
    extra = generate_synthetic(60, dim, 5)
    extra[:5] = x[100:105]  # copies of listed rows under new ids (the queries below include three of them)
    new = np.concatenate([np.arange(n, n + 40), np.arange(0, 20)]).astype(np.int64)  # the last 20 shadow ids 0..19
    idx.add_labels(new, extra)
    assert idx.delete(str(n + 7))
    q = np.concatenate([generate_synthetic(200, dim, 7), x[100:103]])
    opts = SearchOptions(nprobe=4)
    with _env(PYR_PQ_MFMA=0):
        ref = idx.search_batch(q, 10, opts)
    for env in ({}, {"PYR_FILTER_CERR": "1e15"}):
        with _env(**env):
            got, ph = _profiled(hiplib, lambda: idx.search_batch(q, 10, opts))
        assert ph[PH_SAMPLE][0] > 0, "the pq32 path did not run"
        np.testing.assert_array_equal(got[2], ref[2])
        _same(got, ref)
    gcb, gcodes, off, labels, live = idx.pq_state()
    cents = idx.centroids_array()
    bl = np.array([lab != n + 7 for lab in new.tolist()], np.uint8)
    for i in list(range(0, 200, 37)) + [200, 201, 202]:
        os_, ok = oracle.ivfpq_search(q[i], 10, cents, gcodes, off, gcb, live, buf=extra, buf_live=bl, nprobe=4)
        exp = [new[k - oracle.BUFKEY] if k >= oracle.BUFKEY else labels[k] for k in ok]
        np.testing.assert_array_equal(got[1][i][: len(exp)], exp)
        assert np.array_equal(got[0][i][: len(os_)].view(np.uint32), os_.view(np.uint32))


# dsub 32 / 8 / 4 / 16, M = 12 (the 8-lane ADC groups' short last round) and P1's geometry
@pytest.mark.parametrize("dim,m", [(128, 4), (128, 16), (128, 32), (256, 16), (96, 12), (768, 96)])
def test_pq32_large_k_deep_refine(hiplib, oracle, dim, m):
    """k > 60: the matrix-core scan emits at depth K1 = 128 / 256 / 512 and the deep refine
    (pq_deep_refine_kernel) selects, scores by the reference's ADC sum and certifies; what fails re-runs on
    the LUT scan.  Equal to the LUT scan bit for bit at k = 61 .. 256 (as the certificates fall and with all
    forced to fail), and to the oracle."""
    from pyrope_amd import SearchOptions, generate_synthetic
    n = 6000 if dim <= 256 else 3000
    idx, _ = _build(dim, m, n, 12)
    q = generate_synthetic(700, dim, 99)
    opts = SearchOptions(nprobe=5)
    cb, codes, off, labels, live = idx.pq_state()
    cents = idx.centroids_array()
    for k in (61, 100, 200, 256):
        with _env(PYR_PQ_MFMA=0):
            ref = idx.search_batch(q, k, opts)
        got, ph = _profiled(hiplib, lambda: idx.search_batch(q, k, opts))
        assert ph[PH_SAMPLE][0] > 0, "the pq32 path did not run"
        assert ph[PH_FALLBACK][1] < len(q), "no query certified by the deep refine"
        np.testing.assert_array_equal(got[2], ref[2])
        _same(got, ref)
        with _env(PYR_FILTER_CERR="1e15"):
            forced, ph = _profiled(hiplib, lambda: idx.search_batch(q, k, opts))
        assert ph[PH_FALLBACK][1] == len(q)
        _same(forced, ref)
        for i in range(0, len(q), 233):
            os_, ok = oracle.ivfpq_search(q[i], k, cents, codes, off, cb, live, metric=0, nprobe=5)
            np.testing.assert_array_equal(got[1][i][: len(ok)], labels[ok])
            assert np.array_equal(got[0][i][: len(os_)].view(np.uint32), os_.view(np.uint32))
    with _env(PYR_DEEP_REFINE=0):  # the A/B knob: k > 60 back on the LUT scan
        off_run, ph = _profiled(hiplib, lambda: idx.search_batch(q, 100, opts))
    assert ph[PH_SAMPLE][0] == 0
    with _env(PYR_PQ_MFMA=0):
        _same(off_run, idx.search_batch(q, 100, opts))


def test_pq32_large_k_with_buffer_rows(hiplib):
    """k > 60 with rows added after Build: the deep pq32 answer merged with the buffer's exact top k."""
    from pyrope_amd import SearchOptions, generate_synthetic
    n, dim, m = 5000, 128, 16
    idx, x = _build(dim, m, n, 12)
    extra = generate_synthetic(80, dim, 5)
    extra[:5] = x[100:105]
    idx.add_labels(np.arange(n, n + 80, dtype=np.int64), extra)
    q = np.concatenate([generate_synthetic(300, dim, 7), x[100:103]])
    opts = SearchOptions(nprobe=4)
    for k in (100, 200):
        with _env(PYR_PQ_MFMA=0):
            ref = idx.search_batch(q, k, opts)
        got, ph = _profiled(hiplib, lambda: idx.search_batch(q, k, opts))
        assert ph[PH_SAMPLE][0] > 0
        np.testing.assert_array_equal(got[2], ref[2])
        _same(got, ref)
