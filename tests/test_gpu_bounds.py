"""The stream filter's per-row upper bound, row by row.

Every result of the fp16 stream scans is exact because of one property: the score a row is emitted with,
approx + E_row + E_pair (stream_ub_terms, sample16.hip), is at least the reference's own fp32
score of that row (VectorMath.cs:188-253 for FLAT's Unsafe forms, :8-70 for IVF's safe forms, the ADC sum of
IvfPqVectorIndex.cs:182-194 for IVF_PQ).  The certificate (k-th exact score > the K1-th bound) is only as
sound as that inequality, and end-to-end tests would show a too-tight constant only as a rare id mismatch.
Here the scans run with PYR_STREAM_EMIT_ALL=1 (no sampled threshold: every visible row of the scanned lists
is emitted) and a candidate capacity above the rows a query scans; pyr_index_debug_candidates returns every
emitted (bound, label), and the test checks bound >= the oracle's exact score for EVERY row, over uniform,
Gaussian-mixture, offset (+100), wide-range (1e-3 .. 1e3, both signs) and near-duplicate data, d = 96 / 128 /
768, L2 / IP / Cosine on FLAT, L2 / IP on IVF and the IVF_PQ bound (d = 128 / 768).  The slack of each
constant is measured by scripts/bound_slack.py (profiles/r5_bounds/).
"""
import ctypes as C
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

U = 2.0 ** -24
KINDS = ["uniform", "mixture", "offset", "wide", "neardup"]


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


def data(kind, n, d, seed):
    rng = np.random.default_rng(seed)
    if kind == "uniform":
        x = rng.random((n, d))
    elif kind == "mixture":
        c = rng.standard_normal((16, d)) * 4
        x = c[rng.integers(0, 16, n)] + rng.standard_normal((n, d))
    elif kind == "offset":
        x = rng.random((n, d)) + 100.0
    elif kind == "wide":
        x = rng.choice([-1.0, 1.0], (n, d)) * 10.0 ** rng.uniform(-3, 3, (n, d))
    elif kind == "neardup":
        base = rng.random(((n + 7) // 8, d))
        x = np.repeat(base, 8, axis=0)[:n] + 1e-4 * rng.standard_normal((n, d))
    else:
        raise ValueError(kind)
    return np.ascontiguousarray(x, dtype=np.float32)


def emitted(hiplib, idx, q, k, opts, nq_cap):
    """(bounds [nq][cap], labels, counts) of every row the stream scan emitted for queries q"""
    nq = len(q)
    with _env(PYR_STREAM_EMIT_ALL=1, PYR_STREAM_CAP=nq_cap):
        idx.search_batch(q, k, opts)
    ub = np.empty((nq, nq_cap), np.float32)
    lab = np.empty((nq, nq_cap), np.int64)
    cnt = np.empty(nq, np.int32)
    rc = hiplib.pyr_index_debug_candidates(idx._h, nq, nq_cap, ub.ctypes.data_as(C.c_void_p),
                                           lab.ctypes.data_as(C.c_void_p), cnt.ctypes.data_as(C.c_void_p))
    assert rc == 0, hiplib.pyr_last_error()
    assert (cnt <= nq_cap).all()
    return ub, lab, cnt


def margins(ub, lab, cnt, exact_of, transform=None):
    """per query: (labels emitted, bound - exact of each) -- bound in the certificate's form (transform)"""
    out = []
    for i in range(len(cnt)):
        b, l = ub[i, :cnt[i]], lab[i, :cnt[i]]
        keep = l >= 0
        b, l = b[keep], l[keep]
        e = exact_of(i)[l]
        lhs = transform(b) if transform else b.astype(np.float64)
        out.append((l, lhs - e.astype(np.float64), e))
    return out


def check_rows(ub, lab, cnt, exact_of, expect_rows, transform=None):
    """every emitted row's bound >= its exact score; every expected row emitted once; returns the smallest
    margin (bound - exact) relative to max(1, |exact|)"""
    worst = np.inf
    for i, (l, m, e) in enumerate(margins(ub, lab, cnt, exact_of, transform)):
        bad = ~(m >= 0)
        assert not bad.any(), f"query {i}: {int(bad.sum())} rows with bound < exact, e.g. label {l[bad][0]} " \
                              f"margin {m[bad][0]!r} exact {e[bad][0]!r}"
        got = np.unique(l)
        assert len(got) == len(l), "a row was emitted twice"
        np.testing.assert_array_equal(got, np.sort(expect_rows(i)))
        worst = min(worst, float(np.min(m / np.maximum(1.0, np.abs(e)))))
    return worst


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("d", [96, 128, 768])
@pytest.mark.parametrize("metric", [0, 1, 2])
def test_flat_bounds(hiplib, oracle, kind, d, metric):
    from pyrope_amd import BruteForceVectorIndex
    n, nq = 1500, 6
    x = data(kind, n, d, 1)
    q = data(kind, nq, d, 2)
    idx = BruteForceVectorIndex(d, metric)
    idx.add_labels(np.arange(n, dtype=np.int64), x, track_ids=False)
    ub, lab, cnt = emitted(hiplib, idx, q, 10, None, 2048)
    live = np.ones(n, np.uint8)

    def exact_of(i):  # BruteForceVectorIndex.Search's score of every row (the Unsafe forms)
        s, kk = oracle.bf_search(x, live, metric, q[i], n)
        out = np.empty(n, np.float32)
        out[kk] = s
        return out
    tr = None
    if metric == 2:  # the Cosine certificate's form (filter.hip merge_refine_kernel): bound in unit-row L2
        tr = lambda b: 1.0 + 0.5 * b.astype(np.float64) + (2.0 * d + 256.0) * U
    worst = check_rows(ub, lab, cnt, exact_of, lambda i: np.arange(n), tr)
    print(f"\n[bound] FLAT {kind} d={d} metric={metric}: min relative margin {worst:.3g}")
    idx.close()


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("d", [96, 128, 768])
@pytest.mark.parametrize("metric", [0, 1])
def test_ivf_bounds(hiplib, oracle, kind, d, metric):
    from pyrope_amd import IvfFlatVectorIndex, SearchOptions
    n, nq, nl, P = 3000, 6, 8, 3
    x = data(kind, n, d, 3)
    q = data(kind, nq, d, 4)
    idx = IvfFlatVectorIndex(d, metric, n_list=nl)
    idx.add_labels(np.arange(n, dtype=np.int64), x, track_ids=False)
    idx.build()
    opts = SearchOptions(nprobe=P)
    ub, lab, cnt = emitted(hiplib, idx, q, 10, opts, 4096)
    cents = idx.centroids_array()
    off, labels, live = idx.ivf_layout()
    one = np.array([0, n], np.int64)

    def exact_of(i):  # IvfFlatVectorIndex.Search's score (the safe forms) of every row
        s, kk = oracle.ivf_search(q[i], n, cents[:1], x, one, metric=metric, nprobe=1)
        out = np.empty(n, np.float32)
        out[kk] = s
        return out

    def rows_of(i):  # the rows of the query's probed lists
        pr = oracle.ivf_probe(q[i], cents, P, metric=metric)
        return np.concatenate([labels[off[l]:off[l + 1]][live[off[l]:off[l + 1]] != 0] for l in pr])
    worst = check_rows(ub, lab, cnt, exact_of, rows_of)
    print(f"\n[bound] IVF {kind} d={d} metric={metric}: min relative margin {worst:.3g}")
    idx.close()


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("d,m", [(128, 16), (128, 4), (768, 96)])
def test_pq_bounds(hiplib, oracle, kind, d, m):
    from pyrope_amd import IvfPqVectorIndex, SearchOptions
    n, nq, nl, P = 3000, 6, 8, 3
    x = data(kind, n, d, 5)
    q = data(kind, nq, d, 6)
    idx = IvfPqVectorIndex(d, 0, m=m, k=64, n_list=nl)
    idx.add_labels(np.arange(n, dtype=np.int64), x)
    idx.build()
    opts = SearchOptions(nprobe=P)
    ub, lab, cnt = emitted(hiplib, idx, q, 10, opts, 4096)
    cb, codes, off, labels, live = idx.pq_state()
    cents = idx.centroids_array()

    def exact_of(i):  # the ADC sum (IvfPqVectorIndex.cs:182-194) of every row of the probed lists
        s, kk = oracle.ivfpq_search(q[i], n, cents, codes, off, cb, live, metric=0, nprobe=P)
        out = np.full(n, np.inf, np.float32)  # rows outside the probed lists: never emitted
        out[labels[kk]] = s
        return out

    def rows_of(i):
        pr = oracle.ivf_probe(q[i], cents, P, metric=0)
        return np.concatenate([labels[off[l]:off[l + 1]][live[off[l]:off[l + 1]] != 0] for l in pr])
    worst = check_rows(ub, lab, cnt, exact_of, rows_of)
    print(f"\n[bound] IVF_PQ {kind} d={d} m={m}: min relative margin {worst:.3g}")
    idx.close()
