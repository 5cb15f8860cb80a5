"""8-bit search mode of the FLAT index (BruteForceVectorIndex.EnableQuantization) on the GPU.

Reference: Vector/ScalarQuantizer.cs:23-62, Vector/VectorMath.cs:441-681 (L2Squared8Bit,
DotProduct8Bit), Vector/BruteForceVectorIndex.cs:25-40, :166-178, :200-211, :296-336.  Scores
are exact integers converted to float, so the GPU must equal the oracle bit for bit.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_scalar_quantize_matches_oracle(hiplib, oracle):
    from pyrope_amd.vector import scalar_quantize
    rng = np.random.default_rng(3)
    x = rng.normal(size=(300, 77)).astype(np.float32) * 10
    x[0] = 1.5                                    # range 0 -> all zeros (:46-50)
    x[1] = np.linspace(0, 1, 77, dtype=np.float32)
    x[2, :4] = [0.0, 0.5, 1.0, 0.25]              # normalized 127.5 -> 128 (ties to even)
    x[2, 4:] = 0.5
    x[3] = -x[3]
    got = scalar_quantize(x)
    for i in range(len(x)):
        ref, _, _ = oracle.scalar_quantize(x[i])
        np.testing.assert_array_equal(got[i], ref)


def _bf(dim, metric, x, quant_from=0):
    from pyrope_amd import BruteForceVectorIndex
    idx = BruteForceVectorIndex(dim, metric)
    if quant_from > 0:
        idx.add_labels(np.arange(quant_from, dtype=np.int64), x[:quant_from])  # written with quantization off
    idx.enable_quantization = True
    idx.add_labels(np.arange(quant_from, len(x), dtype=np.int64), x[quant_from:])
    return idx


@pytest.mark.parametrize("metric", [0, 1, 2])
@pytest.mark.parametrize("dim,k", [(128, 10), (37, 1), (200, 64), (16, 33), (3, 5), (300, 10), (512, 7)])
def test_quantized_search_matches_oracle(hiplib, oracle, metric, dim, k):
    from pyrope_amd import generate_synthetic
    n = 5000
    x = generate_synthetic(n, dim, 42)
    q = generate_synthetic(40, dim, 1337)
    idx = _bf(dim, metric, x, quant_from=300)  # the first 300 rows have no codes: skipped
    s, lab, cnt = idx.search_batch(q, k)
    has_q = np.ones(n, np.uint8)
    has_q[:300] = 0
    for i in range(len(q)):
        os_, ok = oracle.bf_search_sq8(x, None, has_q, metric, q[i], k)
        assert cnt[i] == len(ok)
        np.testing.assert_array_equal(lab[i][: cnt[i]], ok)
        assert np.array_equal(s[i][: cnt[i]].view(np.uint32), os_.view(np.uint32))


def test_quantized_search_deletes_upserts_max_scans(hiplib, oracle):
    from pyrope_amd import SearchOptions, generate_synthetic
    n, dim = 3000, 64
    x = generate_synthetic(n, dim, 5)
    q = generate_synthetic(20, dim, 6)
    idx = _bf(dim, 0, x)
    live = np.ones(n, np.uint8)
    has_q = np.ones(n, np.uint8)
    for d in range(0, n, 11):
        idx.delete(str(d))
        live[d] = 0
    idx.enable_quantization = False
    for u in range(5, n, 97):  # upsert with quantization off: the slot loses its codes (:206-210)
        if u % 11 == 0:
            continue  # (a deleted id would be re-added at a new slot)
        idx.upsert(str(u), x[u])
        live[u] = 1
        has_q[u] = 0
    idx.enable_quantization = True
    for ms in [None, 0, 1, 700]:
        s, lab, cnt = idx.search_batch(q, 10, SearchOptions(max_scans=ms))
        for i in range(len(q)):
            os_, ok = oracle.bf_search_sq8(x, live, has_q, 0, q[i], 10, max_scans=-1 if ms is None else ms)
            np.testing.assert_array_equal(lab[i][: cnt[i]], ok)
            assert np.array_equal(s[i][: cnt[i]].view(np.uint32), os_.view(np.uint32))


def test_quantization_off_uses_float_path(hiplib, oracle):
    from pyrope_amd import generate_synthetic
    x = generate_synthetic(2000, 32, 8)
    q = generate_synthetic(5, 32, 9)
    idx = _bf(32, 0, x)
    idx.enable_quantization = False
    s, lab, cnt = idx.search_batch(q, 10)
    for i in range(len(q)):
        os_, ok = oracle.bf_search(x, None, 0, q[i], 10)
        np.testing.assert_array_equal(lab[i], ok)


# ---- ScalarQuantizerTests.cs:10-68, restated as written ----
def test_sq_quantize_and_dequantize_round_trip(hiplib):  # :10-30
    from pyrope_amd import ScalarQuantizer
    original = np.array([0.0, 0.5, 1.0, -1.0], np.float32)
    quantized, vmin, vmax = ScalarQuantizer.quantize(original)
    assert len(quantized) == len(original)
    assert vmin == -1.0 and vmax == 1.0
    reconstructed = ScalarQuantizer.dequantize(quantized, vmin, vmax)
    for i in range(len(original)):
        assert abs(original[i] - reconstructed[i]) <= 0.02


def test_sq_quantize_handles_flat_vector(hiplib):  # :32-45
    from pyrope_amd import ScalarQuantizer
    original = np.array([0.5, 0.5, 0.5], np.float32)
    quantized, vmin, vmax = ScalarQuantizer.quantize(original)
    assert vmin == 0.5 and vmax == 0.5
    assert all(b == 0 for b in quantized)
    reconstructed = ScalarQuantizer.dequantize(quantized, vmin, vmax)
    assert all(f == 0.5 for f in reconstructed)


def test_sq_quantize_span_overload_works(hiplib):  # :47-60
    from pyrope_amd import ScalarQuantizer
    original = np.array([0.0, 1.0], np.float32)
    dest = np.zeros(2, np.uint8)
    vmin, vmax = ScalarQuantizer.quantize_into(original, dest)
    assert vmin == 0.0 and vmax == 1.0
    assert dest[0] == 0 and dest[1] == 255
