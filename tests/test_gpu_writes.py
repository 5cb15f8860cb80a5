"""Write-path corner cases: a label repeated inside one batch.

The reference applies Upsert calls one at a time (BruteForceVectorIndex.cs:181-222,
IvfFlatVectorIndex.cs:39-59), so when one batch repeats an id the LAST vector wins and the
id keeps the slot its first occurrence got.  The library must not scatter several rows into
one slot concurrently.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _vecs(n, d, seed):
    return np.random.default_rng(seed).random((n, d), dtype=np.float32)


@pytest.mark.parametrize("n", [3, 5000])
def test_flat_upsert_batch_last_write_wins(hiplib, n):
    from pyrope_amd import BruteForceVectorIndex
    d = 64
    x = _vecs(n, d, 1)
    ids = [f"id{i}" for i in range(n)]
    ids[-1] = "id0"  # the first id again, last in the batch
    idx = BruteForceVectorIndex(d, 0)
    idx.upsert_batch(ids, x)
    rows = idx.scan()
    assert [r[0] for r in rows] == [f"id{i}" for i in range(n - 1)]  # slot order = first occurrence
    np.testing.assert_array_equal(rows[0][1], x[-1])  # the last vector
    res = idx.search(x[-1], 1)
    assert res[0].id == "id0" and res[0].score == 0.0
    assert idx.get_stats().count == n - 1


def test_flat_upsert_batch_repeats_an_existing_id(hiplib):
    from pyrope_amd import BruteForceVectorIndex
    d = 32
    x = _vecs(4, d, 2)
    idx = BruteForceVectorIndex(d, 0)
    idx.add("a", x[0])
    idx.upsert_batch(["a", "b", "a"], x[1:4])
    rows = dict(idx.scan())
    np.testing.assert_array_equal(rows["a"], x[3])
    np.testing.assert_array_equal(rows["b"], x[2])


def test_flat_add_batch_repeat_is_a_duplicate(hiplib):
    from pyrope_amd import BruteForceVectorIndex, InvalidOperationException
    idx = BruteForceVectorIndex(8, 0)
    with pytest.raises(InvalidOperationException):
        idx.add_batch(["a", "a"], _vecs(2, 8, 3))
    assert idx.get_stats().count == 0


@pytest.mark.parametrize("n", [3, 6000])
def test_ivf_add_batch_last_write_wins(hiplib, n):
    from pyrope_amd import IvfFlatVectorIndex
    d = 32
    x = _vecs(n, d, 4)
    ids = [f"v{i}" for i in range(n)]
    ids[-1] = "v1"
    idx = IvfFlatVectorIndex(d, 0, n_list=4)
    idx.add_batch(ids, x)  # IVF Add == buffer upsert (IvfFlatVectorIndex.cs:39-59)
    assert idx.get_stats().count == n - 1
    res = idx.search(x[-1], 1)
    assert res[0].id == "v1" and res[0].score == 0.0
    idx.build()
    res = idx.search(x[-1], 1)
    assert res[0].id == "v1" and res[0].score == 0.0
    assert idx.get_stats().count == n - 1


def test_new_ids_after_caller_labels_do_not_collide(hiplib):
    """add_labels with sparse labels, then a new id through add."""
    from pyrope_amd import BruteForceVectorIndex
    d = 16
    idx = BruteForceVectorIndex(d, 0)
    x = _vecs(4, d, 5)
    idx.add_labels(np.array([0, 2, 4], np.int64), x[:3])
    idx.add("fresh", x[3])  # must not reuse label 3 or any taken label
    assert idx.get_stats().count == 4
    assert idx.search(x[3], 1)[0].id == "fresh"
    assert idx.search(x[1], 1)[0].id == "2"
