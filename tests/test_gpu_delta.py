"""DeltaVectorIndex (head/tail composite) and the registry factory over GPU-backed indexes.

Restates tests/Pyrope.GarnetServer.Tests/Vector/DeltaVectorIndexTests.cs,
Services/VectorIndexRegistryConfigTests.cs and VectorIndexRegistryTests.cs, plus the
compaction path DeltaVectorIndex.Build (DeltaVectorIndex.cs:124-158) through
BruteForceVectorIndex.Scan (BruteForceVectorIndex.cs:250-273, pyr_index_scan).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _bf(dim=2):
    from pyrope_amd import BruteForceVectorIndex
    return BruteForceVectorIndex(dim, 0)


def _delta():
    from pyrope_amd import DeltaVectorIndex
    head, tail = _bf(), _bf()
    return DeltaVectorIndex(head, tail), head, tail


def test_add_writes_to_head(hiplib):  # :23-36
    d, head, tail = _delta()
    d.add("1", [1, 0])
    r = head.search([1, 0], 1)
    assert len(r) == 1 and r[0].id == "1"
    assert tail.search([1, 0], 1) == []


def test_search_merges_results(hiplib):  # :38-50
    d, head, tail = _delta()
    head.add("head1", [1, 0])
    tail.add("tail1", [0, 1])
    ids = {r.id for r in d.search([1, 0], 10)}
    assert ids == {"head1", "tail1"}


def test_search_head_overrides_tail(hiplib):  # :52-66
    d, head, tail = _delta()
    tail.add("doc1", [100, 100])
    head.add("doc1", [1, 0])
    r = d.search([1, 0], 10)
    assert len(r) == 1 and r[0].id == "doc1" and abs(r[0].score) < 1e-3


def test_delete_propagates_to_both(hiplib):  # :68-78
    d, head, tail = _delta()
    head.add("doc1", [1, 0])
    tail.add("doc1", [1, 0])
    d.delete("doc1")
    assert d.search([1, 0], 10) == []


def test_get_centroids_ivf_tail(hiplib):  # :80-95
    from pyrope_amd import DeltaVectorIndex, IvfFlatVectorIndex
    head, tail = _bf(), IvfFlatVectorIndex(2, 0, n_list=2)
    d = DeltaVectorIndex(head, tail)
    tail.add("a1", [0.1, 0.1])
    tail.add("b1", [10, 10])
    tail.build()
    c = d.get_centroids()
    assert c is not None and len(c) > 0


def test_get_centroids_bf_tail_is_none(hiplib):  # :97-104
    d, _, _ = _delta()
    assert d.get_centroids() is None


def test_scan_live_rows_in_slot_order(hiplib):
    from pyrope_amd import generate_synthetic
    x = generate_synthetic(50, 16, 5)
    bf = _bf(16)
    for i in range(50):
        bf.add(f"id{i}", x[i])
    for i in range(0, 50, 3):
        bf.delete(f"id{i}")
    bf.upsert("id4", x[0])  # in place (:193-210): keeps slot 4
    got = bf.scan()
    keep = [i for i in range(50) if i % 3 != 0]
    assert [g[0] for g in got] == [f"id{i}" for i in keep]
    for (gid, v), i in zip(got, keep):
        np.testing.assert_array_equal(v, x[0] if i == 4 else x[i])


@pytest.mark.parametrize("tail_kind", ["bf", "ivf"])
def test_build_compacts_head_into_tail(hiplib, oracle, tail_kind):
    from pyrope_amd import DeltaVectorIndex, IvfFlatVectorIndex, SearchOptions, generate_synthetic
    x = generate_synthetic(600, 32, 9)
    head = _bf(32)
    tail = _bf(32) if tail_kind == "bf" else IvfFlatVectorIndex(32, 0, n_list=8)
    d = DeltaVectorIndex(head, tail)
    for i in range(400):
        d.add(str(i), x[i])
    d.build()
    assert head.get_stats().count == 0 and head.scan() == []
    assert tail.get_stats().count == 400
    for i in range(400, 600):  # fresh writes land in the head again
        d.add(str(i), x[i])
    q = generate_synthetic(5, 32, 10)
    opts = SearchOptions(nprobe=8)
    for qi in q:
        got = d.search(qi, 10, opts)
        # head: BruteForce (*Unsafe form) over rows 400..599; tail: every row 0..399 (nprobe = nlist),
        # BruteForce -> *Unsafe form, IVF_FLAT -> the safe 1-accumulator form (IvfFlatVectorIndex.cs:355)
        hs, hk = oracle.bf_search(x[400:], None, 0, qi, 10)
        if tail_kind == "bf":
            ts, tk = oracle.bf_search(x[:400], None, 0, qi, 10)
        else:
            sc = np.array([-oracle.l2sq(qi, x[i]) for i in range(400)], np.float32)
            tk = np.argsort(-sc, kind="stable")[:10]
            ts = sc[tk]
        merged = {str(j): float(s) for s, j in zip(ts, tk)}
        merged.update({str(j + 400): float(s) for s, j in zip(hs, hk)})
        exp = sorted(merged.items(), key=lambda kv: -kv[1])[:10]
        assert [r.id for r in got] == [e[0] for e in exp]
        assert [r.score for r in got] == [e[1] for e in exp]


def test_registry_config(hiplib):  # VectorIndexRegistryConfigTests.cs
    from pyrope_amd import DeltaVectorIndex, IvfFlatVectorIndex, IvfPqVectorIndex, VectorIndexRegistry
    reg = VectorIndexRegistry()
    d = reg.get_or_create("tenant1", "index_ivf_500", 128, 0, "IVF_FLAT", {"nlist": 500})
    assert isinstance(d, DeltaVectorIndex) and isinstance(d.tail, IvfFlatVectorIndex) and d.tail.n_list == 500
    d2 = reg.get_or_create("tenant1", "index_default", 128, 0)
    assert d2.tail.n_list == 100
    d3 = reg.get_or_create("t", "pq", 16, 0, "ivf_pq", {"m": "8", "k": 16, "nlist": " 4 "})
    assert isinstance(d3.tail, IvfPqVectorIndex) and (d3.tail.m, d3.tail.k, d3.tail.n_list) == (8, 16, 4)
    d4 = reg.get_or_create("t", "weird", 8, 0, "SOMETHING")  # unknown algo -> IVF_FLAT (:103-107)
    assert isinstance(d4.tail, IvfFlatVectorIndex)
    from pyrope_amd import ArgumentException
    with pytest.raises(ArgumentException):
        reg.get_or_create("tenant1", "index_default", 64, 0)


def test_registry_epoch(hiplib):  # VectorIndexRegistryTests.cs
    from pyrope_amd import VectorIndexRegistry
    reg = VectorIndexRegistry()
    reg.get_or_create("tenant", "index", 2, 0)
    assert reg.get_epoch("tenant", "index") == 0
    reg.increment_epoch("tenant", "index")
    reg.increment_epoch("tenant", "index")
    assert reg.get_epoch("tenant", "index") == 2
    assert reg.increment_epoch("tenant", "missing") == 0
