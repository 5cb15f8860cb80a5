"""The filter certificate under adversarial data.

The stream scans (scan.hip; FLAT and IVF_FLAT) rank rows by fp16 approximations and emit every row whose
upper bound (approximation + its share of the error bound, stream_ub_terms) reaches the query's
threshold; the refine takes the reference's exact scores of the best 16 (then 64) and certifies the top k
only if the k-th exact score exceeds the 16th (64th) bound.  Here a query sits at the centre of a shell of
80 rows whose exact scores differ by ~1e-6 -- far inside the fp16 error (~1e-2 at these norms) -- so the
approximations cannot order them, both certificates must fail for that query, and the device-side exact
re-run must return the oracle's ids and score bits anyway.  The profiler counts the re-run queries
(phase 8), so the tests also prove the certificate failed rather than passed by luck.

Metrics: L2 (a shell of radii r0 (1 + i 2^-20)), IP (rows with dot products a0 (1 + i 2^-20) |q|, each
plus an orthogonal component), Cosine (angles off the query that grow by ~1e-6).
"""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

D, N, SHELL, K = 128, 20000, 80, 10


def _shell(metric, seed=11):
    """background rows, the shell rows, the adversarial query"""
    from pyrope_amd import generate_synthetic
    rng = np.random.default_rng(seed)
    x = generate_synthetic(N, D, 42).astype(np.float32)
    q = generate_synthetic(1, D, 7)[0].astype(np.float64)
    u = rng.standard_normal((SHELL, D))
    u /= np.linalg.norm(u, axis=1, keepdims=True)
    step = 1.0 + np.arange(SHELL) * 2.0 ** -20
    if metric == 0:    # L2: a shell of nearly equal radii around q
        rows = q + 0.5 * step[:, None] * u
    elif metric == 1:  # IP: nearly equal q.x, an orthogonal part of norm 1 each
        qh = q / np.linalg.norm(q)
        w = u - (u @ qh)[:, None] * qh
        w /= np.linalg.norm(w, axis=1, keepdims=True)
        rows = (6.0 * step)[:, None] * qh + w
    else:              # Cosine: nearly equal angles to q, norms spread over a decade
        qh = q / np.linalg.norm(q)
        w = u - (u @ qh)[:, None] * qh
        w /= np.linalg.norm(w, axis=1, keepdims=True)
        th = 0.05 * step
        rows = (np.cos(th)[:, None] * qh + np.sin(th)[:, None] * w) * np.linspace(0.5, 5.0, SHELL)[:, None]
    x[rng.choice(N, SHELL, replace=False)] = rows.astype(np.float32)
    qs = np.concatenate([q[None, :], generate_synthetic(15, D, 1337)]).astype(np.float32)
    return x, qs


def _reruns(lib, run):
    """queries the exact re-run took (profiler phase 8) while run() executes"""
    lib.pyr_profile_reset()
    lib.pyr_profile_enable(1)
    try:
        out = run()
    finally:
        lib.pyr_profile_enable(0)
    ms, calls, work = C.c_double(), C.c_int64(), C.c_int64()
    lib.pyr_profile_get(8, C.byref(ms), C.byref(calls), C.byref(work))
    return out, work.value


@pytest.mark.parametrize("metric", [0, 1, 2])
def test_ivf_certificate_fails_and_reruns_exactly(hiplib, oracle, metric):
    from pyrope_amd import IvfFlatVectorIndex, SearchOptions
    x, qs = _shell(metric)
    idx = IvfFlatVectorIndex(D, metric, n_list=8)
    idx.add_labels(np.arange(N, dtype=np.int64), x)
    idx.build()
    opts = SearchOptions(nprobe=8)
    (s, l, c), nre = _reruns(hiplib, lambda: idx.search_batch(qs, K, opts))
    off, labels, live = idx.ivf_layout()
    rows = x[np.where(labels >= 0, labels, 0)]
    cents = idx.centroids_array()
    for i in range(len(qs)):
        os_, ok = oracle.ivf_search(qs[i], K, cents, rows, off, live, metric=metric, nprobe=8)
        np.testing.assert_array_equal(l[i], labels[ok])
        assert np.array_equal(s[i].view(np.uint32), os_.astype(np.float32).view(np.uint32))
    assert nre >= 1, "the shell query must fail both certificates and re-run exactly"


@pytest.mark.parametrize("metric", [0, 1])
def test_flat_certificate_fails_and_reruns_exactly(hiplib, oracle, metric):
    from pyrope_amd import BruteForceVectorIndex
    x, qs = _shell(metric)
    idx = BruteForceVectorIndex(D, metric)
    idx.add_labels(np.arange(N, dtype=np.int64), x)
    (s, l, c), nre = _reruns(hiplib, lambda: idx.search_batch(qs, K))
    for i in range(len(qs)):
        os_, ok = oracle.bf_search(x, None, metric, qs[i], K)
        np.testing.assert_array_equal(l[i], ok)
        assert np.array_equal(s[i].view(np.uint32), os_.astype(np.float32).view(np.uint32))
    assert nre >= 1, "the shell query must fail both certificates and re-run exactly"


def test_shell_is_adversarial(oracle):
    """CPU check of the construction: the shell's exact L2 scores around the query are distinct but
    within 1e-4 of each other, while the fp16 rounding of the residual tiles alone moves them by more."""
    x, qs = _shell(0)
    d = ((x.astype(np.float64) - qs[0].astype(np.float64)) ** 2).sum(1)
    near = np.sort(d)[:SHELL]
    assert near[-1] - near[0] < 1e-4 and np.unique(near).size == SHELL
    x16 = x.astype(np.float16).astype(np.float64)
    d16 = ((x16 - qs[0].astype(np.float64)) ** 2).sum(1)
    assert np.abs(d16 - d)[np.argsort(d)[:SHELL]].max() > 1e-4
