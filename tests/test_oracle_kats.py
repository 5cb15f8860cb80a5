"""Pins the CPU oracle (oracle/oracle.c) against the reference's own known-answer tests.

Every test names the reference test it restates (tests/Pyrope.GarnetServer.Tests/Vector/*.cs);
the .NET System.Random pins are the commonly reported BCL outputs.
Runs on CPU only.
"""
import os

import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


# ---- .NET legacy System.Random (BCL; used by Program.cs:251-263 and KMeansUtils.cs:18) ----
def test_net_random_known_outputs(oracle):
    r = oracle.NetRandom(0)
    assert [r.next() for _ in range(3)] == [1559595546, 1755192844, 1649316166]
    r = oracle.NetRandom(42)
    assert r.next_double() == pytest.approx(0.6681064659115423, abs=0)


def test_generator_float_cast(oracle):
    r = oracle.NetRandom(42)
    ref = np.array([r.next_double() for _ in range(16)], dtype=np.float64).astype(np.float32)
    np.testing.assert_array_equal(oracle.generate_vectors(2, 8, 42).reshape(-1), ref)


# ---- VectorMathTests.cs ----
A5 = [1, 2, 3, 4, 5]
B5 = [2, 3, 4, 5, 6]


def test_dot_product_matches_reference(oracle):  # :10-21
    assert oracle.dot(A5, B5) == pytest.approx(70.0, abs=1e-6)


def test_l2_squared_matches_reference(oracle):  # :23-38
    assert oracle.l2sq(A5, B5) == pytest.approx(5.0, abs=1e-6)


def test_compute_norm_matches_reference(oracle):  # :40-50
    assert oracle.norm(A5) == pytest.approx(np.sqrt(55.0), abs=1e-6)


def test_cosine_matches_reference(oracle):  # :52-65
    assert oracle.cosine([1, 0, 0], [0, 1, 0]) == pytest.approx(0.0, abs=1e-6)
    c = [1, 2, 3]
    assert oracle.cosine(c, c) == pytest.approx(1.0, abs=1e-6)


def _ramp(dim):
    a = (np.arange(dim, dtype=np.float32) * np.float32(0.001)).astype(np.float32)
    b = (np.arange(dim, dtype=np.float32) * np.float32(0.0005)).astype(np.float32)
    return a, b


def test_large_vector_matches_reference(oracle):  # :67-83, d = 1037, tolerance 1.0
    a, b = _ramp(1037)
    exp_dot = np.float32(0)
    exp_l2 = np.float32(0)
    for i in range(1037):
        exp_dot = np.float32(exp_dot + a[i] * b[i])
        d = np.float32(a[i] - b[i])
        exp_l2 = np.float32(exp_l2 + d * d)
    assert oracle.dot(a, b) == pytest.approx(float(exp_dot), abs=1.0)
    assert oracle.l2sq(a, b) == pytest.approx(float(exp_l2), abs=1.0)


def test_unsafe_matches_safe(oracle):  # :108-130, within 1e-4
    a, b = _ramp(1037)
    assert oracle.dot_unsafe(a, b) == pytest.approx(oracle.dot(a, b), abs=1e-4)
    assert oracle.l2sq_unsafe(a, b) == pytest.approx(oracle.l2sq(a, b), abs=1e-4)


def test_8bit_exact(oracle):  # :132-155
    assert oracle.l2sq_8bit([10, 20, 255], [12, 18, 250]) == 33
    assert oracle.dot_8bit([10, 5, 2], [2, 4, 100]) == 240


def test_accumulation_structure(oracle):
    """The 4-accumulator *Unsafe form and the 1-accumulator safe form round differently;
    both must equal an explicit restatement of their own lane structure."""
    x = oracle.generate_vectors(2, 128, 7)
    a, b = x[0], x[1]
    d = (a - b).astype(np.float32)
    sq = (d * d).astype(np.float32)
    acc = np.zeros(8, np.float32)
    for i in range(0, 128, 8):
        acc = (acc + sq[i:i + 8]).astype(np.float32)
    h = np.float32((acc[0] + acc[1]) + (acc[2] + acc[3])) + np.float32((acc[4] + acc[5]) + (acc[6] + acc[7]))
    assert np.float32(oracle.l2sq(a, b)) == np.float32(h)
    accs = [np.zeros(8, np.float32) for _ in range(4)]
    for i in range(0, 128, 32):
        for v in range(4):
            accs[v] = (accs[v] + sq[i + 8 * v:i + 8 * v + 8]).astype(np.float32)
    fin = (((accs[0] + accs[1]).astype(np.float32) + accs[2]).astype(np.float32) + accs[3]).astype(np.float32)
    h4 = np.float32((fin[0] + fin[1]) + (fin[2] + fin[3])) + np.float32((fin[4] + fin[5]) + (fin[6] + fin[7]))
    assert np.float32(oracle.l2sq_unsafe(a, b)) == np.float32(h4)


# ---- BruteForceVectorIndexTests.cs ----
def test_bf_cosine_returns_closest(oracle):  # :10-20
    rows = np.array([[1, 0], [0, 1]], np.float32)
    s, k = oracle.bf_search(rows, None, oracle.COS, [1, 0.1], 1)
    assert list(k) == [0]


def test_bf_upsert_semantics(oracle):  # :22-33 (upsert = overwrite slot 0)
    rows = np.array([[0, 2]], np.float32)
    s, k = oracle.bf_search(rows, None, oracle.IP, [0, 1], 1)
    assert list(k) == [0] and s[0] > 1


def test_bf_delete_and_max_scans(oracle):  # :35-46, :56-65
    rows = np.array([[1, 1]], np.float32)
    s, k = oracle.bf_search(rows, np.array([0], np.uint8), oracle.L2, [1, 1], 1)
    assert len(k) == 0
    rows = np.array([[1, 0], [0, 1]], np.float32)
    s, k = oracle.bf_search(rows, None, oracle.IP, [1, 0], 1, max_scans=0)
    assert len(k) == 0


def test_bf_max_scans_counts_live_slots_in_order(oracle):  # BruteForceVectorIndex.cs:341-345
    rows = np.array([[5], [4], [3], [2], [1]], np.float32)
    live = np.array([1, 0, 1, 1, 1], np.uint8)
    s, k = oracle.bf_search(rows, live, oracle.L2, [0], 5, max_scans=2)
    assert sorted(k.tolist()) == [0, 2]


# ---- IvfFlatVectorIndexTests.cs ----
def test_ivf_search_before_build_uses_buffer(oracle):  # :51-66
    buf = np.array([[1, 0], [5, 5]], np.float32)
    s, k = oracle.ivf_search([1, 0], 1, np.zeros((0, 2)), np.zeros((0, 2)), np.zeros(1, np.int64), buf=buf,
                             built=False)
    assert list(k) == [oracle.BUFKEY + 0]


def test_ivf_build_clusters_data(oracle):  # :68-90
    x = np.array([[0.1, 0.1], [0.2, 0.2], [10.1, 10.1], [10.2, 10.2]], np.float32)
    cents, assign = oracle.ivf_build(x, 2, oracle.L2)
    rows, order, off = oracle.lists_from_assign(x, assign, 2)
    s, k = oracle.ivf_search([0, 0], 2, cents, rows, off, nprobe=1)
    assert len(k) == 2
    assert {int(order[i]) for i in k} == {0, 1}


def test_ivf_nprobe_equal_nlist_returns_all(oracle):  # :92-116
    x = np.array([[0, 0], [5, 5], [10, 10]], np.float32)
    cents, assign = oracle.ivf_build(x, 3, oracle.L2)
    rows, order, off = oracle.lists_from_assign(x, assign, 3)
    s, k = oracle.ivf_search([0, 0], 3, cents, rows, off, nprobe=3)
    assert len(k) == 3


# ---- IvfPqVectorIndexTests.cs ----
def test_pq_encode_length(oracle):  # :11-39
    r = oracle.NetRandom(42)
    data = np.array([[r.next_double() for _ in range(16)] for _ in range(100)], np.float32)
    cb = oracle.pq_train(data, 4, 256)
    code = oracle.pq_encode(np.full(16, 0.5, np.float32), cb)
    assert code.shape == (4,)
    assert cb.shape == (4, 100, 4)  # codebook size = min(K, n_train) (KMeansUtils.cs:14)


def test_ivfpq_search_returns_results(oracle):  # :41-67
    r = oracle.NetRandom(123)
    data = np.array([[r.next_double() for _ in range(128)] for _ in range(100)], np.float32)
    cents, assign, cb, codes = oracle.ivfpq_build(data, 4, 16, 256, oracle.L2)
    _, order, off = oracle.lists_from_assign(data, assign, len(cents))
    s, k = oracle.ivfpq_search(np.full(128, 0.5, np.float32), 5, cents, codes[order], off, cb, nprobe=-1)
    assert len(k) == 5


# ---- golden fixtures (tests/golden/make_golden.py) ----
def test_golden_generator(oracle):
    g = np.load(os.path.join(GOLDEN, "generator.npz"))
    np.testing.assert_array_equal(oracle.generate_vectors(2, 8, 42).reshape(-1), g["gen_seed42_first16"])
    np.testing.assert_array_equal(oracle.generate_vectors(2, 8, 1337).reshape(-1), g["gen_seed1337_first16"])
    r = oracle.NetRandom(0)
    assert [r.next() for _ in range(5)] == g["random_seed0_next5"].tolist()


def test_golden_flat(oracle):
    g = np.load(os.path.join(GOLDEN, "flat_d128.npz"))
    x = oracle.generate_vectors(int(g["n"]), int(g["dim"]), int(g["base_seed"]))
    q = oracle.generate_vectors(int(g["nq"]), int(g["dim"]), int(g["query_seed"]))
    for m, name in [(0, "l2"), (1, "ip"), (2, "cos")]:
        for i in range(0, int(g["nq"]), 7):
            s, k = oracle.bf_search(x, None, m, q[i], int(g["k"]))
            np.testing.assert_array_equal(k, g[f"{name}_keys"][i])
            np.testing.assert_array_equal(s.view(np.uint32), g[f"{name}_scores"][i].view(np.uint32))


def test_golden_ivf_flat(oracle):
    g = np.load(os.path.join(GOLDEN, "ivf_flat.npz"))
    x = oracle.generate_vectors(int(g["n"]), int(g["dim"]), 42)
    cents, assign = oracle.ivf_build(x, int(g["nlist"]), 0)
    np.testing.assert_array_equal(cents.view(np.uint32), g["centroids"].view(np.uint32))
    np.testing.assert_array_equal(assign, g["assign"])


def test_golden_ivf_pq(oracle):
    g = np.load(os.path.join(GOLDEN, "ivf_pq.npz"))
    x = oracle.generate_vectors(int(g["n"]), int(g["dim"]), 42)
    cents, assign, cb, codes = oracle.ivfpq_build(x, int(g["nlist"]), int(g["m"]), 256, 0)
    np.testing.assert_array_equal(cb.view(np.uint32), g["codebooks"].view(np.uint32))
    np.testing.assert_array_equal(codes, g["codes"])


# ---- ScalarQuantizer.cs / VectorMath 8-bit (the BruteForce EnableQuantization mode) ----
def test_scalar_quantize_known_answers(oracle):
    c, mn, mx = oracle.scalar_quantize([0.0, 0.5, 1.0, 0.25])  # 127.5 -> 128, 63.75 -> 64
    assert list(c) == [0, 128, 255, 64] and (mn, mx) == (0.0, 1.0)
    c, mn, mx = oracle.scalar_quantize([2.0, 2.0, 2.0])        # range 0 -> zeros (:46-50)
    assert list(c) == [0, 0, 0] and (mn, mx) == (2.0, 2.0)
    c, _, _ = oracle.scalar_quantize([-1.0, 1.0, 0.0])         # 127.5 -> 128
    assert list(c) == [0, 255, 128]


def test_8bit_simd_wrap_semantics(oracle):
    """The x64 SIMD path sums the first n - n % 32 terms in wrapping int32 lanes: identical to
    the exact sum below 33,025 dims, wrapped above (VectorMath.cs:441-564)."""
    rng = np.random.default_rng(0)
    a = rng.integers(0, 256, 1000, dtype=np.uint8)
    b = rng.integers(0, 256, 1000, dtype=np.uint8)
    assert oracle.l2sq_8bit_net(a, b) == oracle.l2sq_8bit(a, b)
    assert oracle.dot_8bit_net(a, b) == oracle.dot_8bit(a, b)
    big = np.full(40000, 255, np.uint8)
    exact = 40000 * 255 * 255
    simd = 40000 - 40000 % 32
    wrapped = ((simd * 65025 + 2**31) % 2**32) - 2**31 + (40000 - simd) * 65025
    assert oracle.dot_8bit(big, big) == exact
    assert oracle.dot_8bit_net(big, big) == wrapped
