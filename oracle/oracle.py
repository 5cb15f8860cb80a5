"""ctypes wrapper over oracle/liboracle.so (the C restatement in oracle.c).

TEST INFRASTRUCTURE ONLY: see oracle/__init__.py.  Every wrapper names the
reference function it restates (paths relative to
/root/reference/src/Pyrope.GarnetServer/).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

L2, IP, COS = 0, 1, 2
BUFKEY = 1 << 31

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "liboracle.so")
_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib_w4():
    """The 4-lane (Arm64 NEON Vector<float>) build of the same restatement: lane-width study only."""
    so = os.path.join(_HERE, "liboracle_w4.so")
    subprocess.run(["make", "-s", "-C", _HERE, "w4"], check=True)
    L = C.CDLL(so)
    _declare(L)
    return L


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO) or os.path.getmtime(_SO) < os.path.getmtime(os.path.join(_HERE, "oracle.c")):
            build()
        _lib = C.CDLL(_SO)
        _declare(_lib)
    return _lib


_f = C.POINTER(C.c_float)
_u8 = C.POINTER(C.c_uint8)
_i32 = C.POINTER(C.c_int32)
_i64 = C.POINTER(C.c_int64)


def _declare(L):
    I32, I64, F, D = C.c_int32, C.c_int64, C.c_float, C.c_double
    sig = {
        "orc_random_init": (None, [C.c_void_p, I32]),
        "orc_random_next": (I32, [C.c_void_p]),
        "orc_random_next_double": (D, [C.c_void_p]),
        "orc_generate_vectors": (None, [I64, I32, I32, _f]),
        "orc_dot": (F, [_f, _f, I32]),
        "orc_l2sq": (F, [_f, _f, I32]),
        "orc_norm": (F, [_f, I32]),
        "orc_cosine": (F, [_f, _f, I32, F, F]),
        "orc_dot_unsafe": (F, [_f, _f, I32]),
        "orc_l2sq_unsafe": (F, [_f, _f, I32]),
        "orc_l2sq_8bit": (I64, [_u8, _u8, I32]),
        "orc_dot_8bit": (I64, [_u8, _u8, I32]),
        "orc_bf_search": (I32, [_f, _u8, I64, I32, I32, _f, I32, I64, _f, _i64]),
        "orc_find_nearest_centroid": (I32, [_f, _f, _f, I32, I32, I32]),
        "orc_kmeans_train": (I32, [_f, I64, I32, I32, I32, I32, I32, _f]),
        "orc_ivf_build": (I32, [_f, I64, I32, I32, I32, _f, _i32]),
        "orc_ivf_search": (I32, [_f, _u8, I64, _f, _u8, _i64, _f, I32, I32, I32, I32, _f, I32, I32, I64, _f, _i64]),
        "orc_pq_train": (I32, [_f, I64, I32, I32, I32, _f]),
        "orc_pq_encode": (None, [_f, I32, I32, I32, _f, _u8]),
        "orc_pq_distance_table": (None, [_f, I32, I32, I32, _f, _f]),
        "orc_ivfpq_build": (I32, [_f, I64, I32, I32, I32, I32, I32, _f, _i32, _f, _i32, _u8]),
        "orc_ivfpq_search": (I32, [_f, _u8, I64, _u8, _u8, _i64, _f, I32, I32, _f, I32, I32, I32, I32, _f, I32, I32, _f, _i64]),
        "orc_ivf_search_batch": (None, [_f, _u8, I64, _f, _u8, _i64, _f, I32, I32, I32, _f, I64, I32, I32, I32, _f, _i64, _i32]),
        "orc_bf_search_batch": (None, [_f, _u8, I64, I32, I32, _f, I64, I32, I32, _f, _i64, _i32]),
        "orc_ivf_probe": (I32, [_f, _f, I32, I32, I32, I32, _i32]),
        "orc_ivf_search_probed": (I32, [_f, _i64, _u8, _i64, _i32, I32, I32, I32, _f, I32, _f, _i64]),
        "orc_ivf_search_batch_idx": (None, [_f, _i64, _u8, _i64, _f, I32, I32, I32, _f, I64, I32, I32, I32, _f, _i64,
                                            _i32]),
        "orc_scalar_quantize": (None, [_f, I32, _u8, _f, _f]),
        "orc_l2sq_8bit_net": (I64, [_u8, _u8, I32]),
        "orc_dot_8bit_net": (I64, [_u8, _u8, I32]),
        "orc_bf_search_sq8": (I32, [_f, _u8, _u8, I64, I32, I32, _f, I32, I64, _f, _i64]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args


def _p(a, ct):
    if a is None:
        return C.cast(None, C.POINTER(ct))
    return a.ctypes.data_as(C.POINTER(ct))


def _f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def _u8a(a):
    return np.ascontiguousarray(a, dtype=np.uint8)


class NetRandom:
    """System.Random(int) legacy generator (BCL)."""

    def __init__(self, seed: int):
        self._state = C.create_string_buffer(58 * 4)
        lib().orc_random_init(self._state, seed)

    def next(self) -> int:
        return lib().orc_random_next(self._state)

    def next_double(self) -> float:
        return lib().orc_random_next_double(self._state)


def generate_vectors(count: int, dim: int, seed: int) -> np.ndarray:
    """Pyrope.Benchmarks/Program.cs:251-263 GenerateRandomVectors."""
    out = np.empty((count, dim), dtype=np.float32)
    lib().orc_generate_vectors(count, dim, seed, _p(out, C.c_float))
    return out


# VectorMath.cs
def dot(a, b):
    a, b = _f32(a), _f32(b)
    return lib().orc_dot(_p(a, C.c_float), _p(b, C.c_float), a.size)


def l2sq(a, b):
    a, b = _f32(a), _f32(b)
    return lib().orc_l2sq(_p(a, C.c_float), _p(b, C.c_float), a.size)


def norm(v):
    v = _f32(v)
    return lib().orc_norm(_p(v, C.c_float), v.size)


def cosine(q, v, qn=None, vn=None):
    q, v = _f32(q), _f32(v)
    qn = norm(q) if qn is None else qn
    vn = norm(v) if vn is None else vn
    return lib().orc_cosine(_p(q, C.c_float), _p(v, C.c_float), q.size, qn, vn)


def dot_unsafe(a, b):
    a, b = _f32(a), _f32(b)
    return lib().orc_dot_unsafe(_p(a, C.c_float), _p(b, C.c_float), a.size)


def l2sq_unsafe(a, b):
    a, b = _f32(a), _f32(b)
    return lib().orc_l2sq_unsafe(_p(a, C.c_float), _p(b, C.c_float), a.size)


def l2sq_8bit(a, b):
    a, b = _u8a(a), _u8a(b)
    return lib().orc_l2sq_8bit(_p(a, C.c_uint8), _p(b, C.c_uint8), a.size)


def dot_8bit(a, b):
    a, b = _u8a(a), _u8a(b)
    return lib().orc_dot_8bit(_p(a, C.c_uint8), _p(b, C.c_uint8), a.size)


def bf_search(rows, live, metric, q, k, max_scans=-1):
    """BruteForceVectorIndex.cs:275-379.  Returns (scores, slot keys)."""
    rows = _f32(rows)
    n, dim = rows.shape
    live = _u8a(np.ones(n) if live is None else live)
    q = _f32(q)
    s = np.empty(max(k, 1), np.float32)
    kk = np.empty(max(k, 1), np.int64)
    c = lib().orc_bf_search(_p(rows, C.c_float), _p(live, C.c_uint8), n, dim, metric, _p(q, C.c_float), k,
                            max_scans, _p(s, C.c_float), _p(kk, C.c_int64))
    return s[:c], kk[:c]


def scalar_quantize(v):
    """ScalarQuantizer.Quantize (ScalarQuantizer.cs:23-62) -> (codes uint8, min, max)."""
    v = _f32(v).reshape(-1)
    out = np.zeros(max(v.size, 1), np.uint8)
    mn, mx = C.c_float(), C.c_float()
    lib().orc_scalar_quantize(_p(v, C.c_float), v.size, _p(out, C.c_uint8), C.byref(mn), C.byref(mx))
    return out[: v.size], mn.value, mx.value


def l2sq_8bit_net(a, b):
    """VectorMath.L2Squared8Bit with the x64 SIMD path's int32 wrap of the vector part."""
    a, b = _u8a(a), _u8a(b)
    return lib().orc_l2sq_8bit_net(_p(a, C.c_uint8), _p(b, C.c_uint8), a.size)


def dot_8bit_net(a, b):
    a, b = _u8a(a), _u8a(b)
    return lib().orc_dot_8bit_net(_p(a, C.c_uint8), _p(b, C.c_uint8), a.size)


def bf_search_sq8(rows, live, has_q, metric, q, k, max_scans=-1):
    """BruteForceVectorIndex.Search with EnableQuantization (:296-336).  Returns (scores, slots)."""
    rows = _f32(rows)
    n, dim = rows.shape
    live = _u8a(np.ones(n) if live is None else live)
    has_q = _u8a(np.ones(n) if has_q is None else has_q)
    q = _f32(q)
    s = np.empty(max(k, 1), np.float32)
    kk = np.empty(max(k, 1), np.int64)
    c = lib().orc_bf_search_sq8(_p(rows, C.c_float), _p(live, C.c_uint8), _p(has_q, C.c_uint8), n, dim, metric,
                                _p(q, C.c_float), k, max_scans, _p(s, C.c_float), _p(kk, C.c_int64))
    return s[:c], kk[:c]


def find_nearest_centroid(v, cents, metric):
    """KMeansUtils.cs:70-93."""
    v, cents = _f32(v), _f32(cents)
    k, dim = cents.shape
    cn = np.array([norm(c) if metric == COS else 0.0 for c in cents], np.float32)
    return lib().orc_find_nearest_centroid(_p(v, C.c_float), _p(cents, C.c_float), _p(cn, C.c_float), k, dim, metric)


def kmeans_train(data, k, metric, max_iter=10, seed=42):
    """KMeansUtils.cs:10-68."""
    data = _f32(data)
    n, dim = data.shape
    out = np.zeros((max(min(max(k, 1), n), 1), dim), np.float32)
    kk = lib().orc_kmeans_train(_p(data, C.c_float), n, dim, k, metric, max_iter, seed, _p(out, C.c_float))
    return out[:kk]


def ivf_build(data, nlist, metric):
    """IvfFlatVectorIndex.cs:111-132 (rows given in uniqueData order)."""
    data = _f32(data)
    n, dim = data.shape
    cents = np.zeros((max(min(nlist, n), 1), dim), np.float32)
    assign = np.zeros(n, np.int32)
    k = lib().orc_ivf_build(_p(data, C.c_float), n, dim, nlist, metric, _p(cents, C.c_float), _p(assign, C.c_int32))
    return cents[:k], assign


def lists_from_assign(data, assign, nlist):
    """Stable list-major layout: lists[c] keeps uniqueData order (IvfFlat.cs:128-132)."""
    order = np.argsort(assign, kind="stable")
    counts = np.bincount(assign, minlength=nlist)
    off = np.zeros(nlist + 1, np.int64)
    off[1:] = np.cumsum(counts)
    return data[order], order, off


def ivf_search(q, k, cents, lrows, list_off, row_live=None, buf=None, buf_live=None, metric=L2,
               nprobe=-1, max_scans=-1, built=True):
    """IvfFlatVectorIndex.cs:147-231.  Returns (scores, keys)."""
    q = _f32(q)
    dim = q.size
    cents = _f32(cents).reshape(-1, dim)
    lrows = _f32(lrows).reshape(-1, dim)
    list_off = np.ascontiguousarray(list_off, np.int64)
    row_live = _u8a(np.ones(len(lrows)) if row_live is None else row_live)
    buf = _f32(np.zeros((0, dim)) if buf is None else buf).reshape(-1, dim)
    buf_live = _u8a(np.ones(len(buf)) if buf_live is None else buf_live)
    s = np.empty(max(k, 1), np.float32)
    kk = np.empty(max(k, 1), np.int64)
    c = lib().orc_ivf_search(_p(buf, C.c_float), _p(buf_live, C.c_uint8), len(buf), _p(lrows, C.c_float),
                             _p(row_live, C.c_uint8), _p(list_off, C.c_int64), _p(cents, C.c_float), len(cents),
                             int(built), dim, metric, _p(q, C.c_float), k, nprobe, max_scans,
                             _p(s, C.c_float), _p(kk, C.c_int64))
    return s[:c], kk[:c]


def pq_train(data, M, K):
    """ProductQuantizer.cs:28-58.  Returns codebooks [M][ksub][sub]."""
    data = _f32(data)
    n, dim = data.shape
    sub = dim // M
    ksub_max = max(min(K, n), 1)
    cb = np.zeros((M, ksub_max, sub), np.float32)
    ksub = lib().orc_pq_train(_p(data, C.c_float), n, dim, M, K, _p(cb, C.c_float))
    return cb[:, :ksub, :].copy() if ksub == ksub_max else cb.reshape(-1)[: M * ksub * sub].reshape(M, ksub, sub)


def pq_encode(v, cb):
    """ProductQuantizer.cs:60-80."""
    v, cb = _f32(v), _f32(cb)
    M, ksub, sub = cb.shape
    code = np.zeros(M, np.uint8)
    lib().orc_pq_encode(_p(v, C.c_float), v.size, M, ksub, _p(cb, C.c_float), _p(code, C.c_uint8))
    return code


def pq_distance_table(q, cb):
    """ProductQuantizer.cs:98-120."""
    q, cb = _f32(q), _f32(cb)
    M, ksub, sub = cb.shape
    t = np.zeros((M, ksub), np.float32)
    lib().orc_pq_distance_table(_p(q, C.c_float), q.size, M, ksub, _p(cb, C.c_float), _p(t, C.c_float))
    return t


def ivfpq_build(data, nlist, M, K, metric):
    """IvfPqVectorIndex.cs:55-116.  Returns (cents, assign, codebooks, codes)."""
    data = _f32(data)
    n, dim = data.shape
    nc_max = max(min(nlist, n), 1)
    cents = np.zeros((nc_max, dim), np.float32)
    assign = np.zeros(n, np.int32)
    ksub_max = max(min(K, n), 1)
    cb = np.zeros(M * ksub_max * (dim // M), np.float32)
    ksub = np.zeros(1, np.int32)
    codes = np.zeros((n, M), np.uint8)
    nc = lib().orc_ivfpq_build(_p(data, C.c_float), n, dim, nlist, M, K, metric, _p(cents, C.c_float),
                               _p(assign, C.c_int32), _p(cb, C.c_float), _p(ksub, C.c_int32), _p(codes, C.c_uint8))
    ks = int(ksub[0])
    return cents[:nc], assign, cb[: M * ks * (dim // M)].reshape(M, ks, dim // M), codes


def ivfpq_search(q, k, cents, codes, list_off, cb, row_live=None, buf=None, buf_live=None, metric=L2,
                 nprobe=-1, built=True):
    """IvfPqVectorIndex.cs:118-212.  codes list-major."""
    q = _f32(q)
    dim = q.size
    cents = _f32(cents).reshape(-1, dim)
    codes = _u8a(codes)
    cb = _f32(cb)
    M, ksub, _ = cb.shape
    list_off = np.ascontiguousarray(list_off, np.int64)
    row_live = _u8a(np.ones(len(codes)) if row_live is None else row_live)
    buf = _f32(np.zeros((0, dim)) if buf is None else buf).reshape(-1, dim)
    buf_live = _u8a(np.ones(len(buf)) if buf_live is None else buf_live)
    s = np.empty(max(k, 1), np.float32)
    kk = np.empty(max(k, 1), np.int64)
    c = lib().orc_ivfpq_search(_p(buf, C.c_float), _p(buf_live, C.c_uint8), len(buf), _p(codes, C.c_uint8),
                               _p(row_live, C.c_uint8), _p(list_off, C.c_int64), _p(cents, C.c_float), len(cents),
                               int(built), _p(cb, C.c_float), M, ksub, dim, metric, _p(q, C.c_float), k, nprobe,
                               _p(s, C.c_float), _p(kk, C.c_int64))
    return s[:c], kk[:c]


def ivf_search_batch(qs, k, cents, lrows, list_off, row_live=None, metric=L2, nprobe=-1, nthreads=1):
    """CPU baseline: one query per worker thread (Program.cs:363-388 concurrency)."""
    qs = _f32(qs)
    nq, dim = qs.shape
    cents, lrows = _f32(cents), _f32(lrows)
    list_off = np.ascontiguousarray(list_off, np.int64)
    row_live = _u8a(np.ones(len(lrows)) if row_live is None else row_live)
    buf = np.zeros((1, dim), np.float32)
    bl = np.zeros(1, np.uint8)
    s = np.full((nq, k), -np.inf, np.float32)
    kk = np.full((nq, k), -1, np.int64)
    cnt = np.zeros(nq, np.int32)
    lib().orc_ivf_search_batch(_p(buf, C.c_float), _p(bl, C.c_uint8), 0, _p(lrows, C.c_float),
                               _p(row_live, C.c_uint8), _p(list_off, C.c_int64), _p(cents, C.c_float), len(cents),
                               dim, metric, _p(qs, C.c_float), nq, k, nprobe, nthreads,
                               _p(s, C.c_float), _p(kk, C.c_int64), _p(cnt, C.c_int32))
    return s, kk, cnt


def bf_search_batch(qs, k, rows, live=None, metric=L2, nthreads=1):
    qs, rows = _f32(qs), _f32(rows)
    nq, dim = qs.shape
    live = _u8a(np.ones(len(rows)) if live is None else live)
    s = np.full((nq, k), -np.inf, np.float32)
    kk = np.full((nq, k), -1, np.int64)
    cnt = np.zeros(nq, np.int32)
    lib().orc_bf_search_batch(_p(rows, C.c_float), _p(live, C.c_uint8), len(rows), dim, metric, _p(qs, C.c_float),
                              nq, k, nthreads, _p(s, C.c_float), _p(kk, C.c_int64), _p(cnt, C.c_int32))
    return s, kk, cnt


def ivf_probe(q, cents, nprobe, metric=L2):
    """IvfFlatVectorIndex.cs:186-198: the first min(nprobe, nlist) lists by (score desc, index asc)."""
    q, cents = _f32(q).reshape(-1), _f32(cents)
    nlist, dim = cents.shape
    out = np.zeros(max(nprobe, 1), np.int32)
    n = lib().orc_ivf_probe(_p(q, C.c_float), _p(cents, C.c_float), nlist, dim, metric, nprobe, _p(out, C.c_int32))
    return out[:n]


def ivf_search_probed(q, k, lrows, list_off, probes, row_live=None, row_idx=None, metric=L2):
    """IvfFlatVectorIndex.cs:200-218 over caller-ranked lists.  Returns (scores, list-major keys)."""
    q, lrows = _f32(q).reshape(-1), _f32(lrows)
    dim = q.size
    list_off = np.ascontiguousarray(list_off, np.int64)
    probes = np.ascontiguousarray(probes, np.int32)
    live = None if row_live is None else _u8a(row_live)
    ridx = None if row_idx is None else np.ascontiguousarray(row_idx, np.int64)
    s = np.empty(max(k, 1), np.float32)
    kk = np.empty(max(k, 1), np.int64)
    c = lib().orc_ivf_search_probed(_p(lrows, C.c_float), _p(ridx, C.c_int64), _p(live, C.c_uint8),
                                    _p(list_off, C.c_int64), _p(probes, C.c_int32), len(probes), dim, metric,
                                    _p(q, C.c_float), k, _p(s, C.c_float), _p(kk, C.c_int64))
    return s[:c], kk[:c]


def ivf_search_batch_idx(qs, k, cents, rows, row_idx, list_off, row_live=None, metric=L2, nprobe=-1, nthreads=1):
    """CPU baseline over base rows + layout labels (no list-major copy): one query per thread."""
    qs, rows, cents = _f32(qs), _f32(rows), _f32(cents)
    nq, dim = qs.shape
    row_idx = np.ascontiguousarray(row_idx, np.int64)
    list_off = np.ascontiguousarray(list_off, np.int64)
    live = None if row_live is None else _u8a(row_live)
    s = np.full((nq, k), -np.inf, np.float32)
    kk = np.full((nq, k), -1, np.int64)
    cnt = np.zeros(nq, np.int32)
    lib().orc_ivf_search_batch_idx(_p(rows, C.c_float), _p(row_idx, C.c_int64), _p(live, C.c_uint8),
                                   _p(list_off, C.c_int64), _p(cents, C.c_float), len(cents), dim, metric,
                                   _p(qs, C.c_float), nq, k, nprobe, nthreads, _p(s, C.c_float), _p(kk, C.c_int64),
                                   _p(cnt, C.c_int32))
    return s, kk, cnt
