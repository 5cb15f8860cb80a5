"""IVectorIndex.Snapshot / Load (IVectorIndex.cs:26-27) through pyr_index_snapshot / pyr_index_load.

Restates the reference's tests IvfFlatVectorIndexTests.cs:119-141 (SnapshotLoad_PreservesState)
and :144-165 (Load_MissingFields_ShouldHandleGracefully), the Delta manifest round trip
(DeltaVectorIndex.cs:160-212), and checks that every index kind searches bit-identically after a
round trip (deletes, upserts, buffer rows shadowing list rows, IVF_PQ codes).
"""
import os
import struct

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _same(a, b):
    (s1, l1, c1), (s2, l2, c2) = a, b
    np.testing.assert_array_equal(c1, c2)
    np.testing.assert_array_equal(l1, l2)
    assert np.array_equal(s1.view(np.uint32), s2.view(np.uint32))


def test_snapshot_load_preserves_state(hiplib, tmp_path):  # IvfFlatVectorIndexTests.cs:119-141
    from pyrope_amd import IvfFlatVectorIndex, VectorMetric
    path = str(tmp_path / "ivf.snap")
    index = IvfFlatVectorIndex(2, VectorMetric.L2, n_list=2)
    index.add("a", [1.0, 0.0])
    index.build()
    index.snapshot(path)
    loaded = IvfFlatVectorIndex(2, VectorMetric.L2, n_list=2)
    loaded.load(path)
    results = loaded.search([1.0, 0.0], 1)
    assert len(results) == 1 and results[0].id == "a"


def _image(path, kind, dim, metric, sections):
    """A hand-written index image (persist.h layout)."""
    with open(path, "wb") as f:
        f.write(b"PYRIDX01" + struct.pack("<iiiiI", 1, kind, dim, metric, len(sections)))
        for tag, payload in sections:
            f.write(struct.pack("<IIQ", tag, 0, len(payload)) + payload + b"\0" * ((8 - len(payload) % 8) % 8))


def test_load_missing_fields_handled_gracefully(hiplib, tmp_path):  # IvfFlatVectorIndexTests.cs:144-165
    """A partial image (not built, empty buffer, no centroids / lists: an "old format") loads to a
    safe empty state.  Like the reference (whose JSON says Metric 1 for an L2 index), the recorded
    metric is not enforced."""
    from pyrope_amd import IvfFlatVectorIndex, VectorMetric
    path = str(tmp_path / "partial.snap")
    _image(path, 1, 2, 1, [(1, b"\0"), (6, b"")])  # T_BUILT = 0, T_BLABELS = []
    index = IvfFlatVectorIndex(2, VectorMetric.L2)
    index.load(path)
    assert index.search([0.0, 0.0], 1) == []
    assert index.get_stats().count == 0


def test_load_errors(hiplib, tmp_path):
    from pyrope_amd import BruteForceVectorIndex, IvfFlatVectorIndex
    from pyrope_amd._lib import ArgumentException, FileNotFoundException, JsonException
    idx = IvfFlatVectorIndex(4, 0, n_list=2)
    with pytest.raises(FileNotFoundException):  # IvfFlatVectorIndex.cs:259
        idx.load(str(tmp_path / "nope"))
    with pytest.raises(ArgumentException):  # BruteForceVectorIndex.cs:60
        idx.snapshot(" ")
    bf = BruteForceVectorIndex(4, 0)
    bf.add("x", [1, 2, 3, 4])
    bf.snapshot(str(tmp_path / "bf"))
    with pytest.raises(JsonException):  # another kind
        idx.load(str(tmp_path / "bf"))
    with pytest.raises(JsonException):  # another dimension
        BruteForceVectorIndex(8, 0).load(str(tmp_path / "bf"))
    (tmp_path / "junk").write_bytes(b"{\"Dimension\": 4}")
    with pytest.raises(JsonException):
        idx.load(str(tmp_path / "junk"))
    assert not os.path.exists(str(tmp_path / "bf.tmp"))  # the temp file was renamed into place


@pytest.mark.parametrize("metric", [0, 1, 2])
def test_flat_round_trip(hiplib, tmp_path, metric):
    from pyrope_amd import BruteForceVectorIndex, SearchOptions, generate_synthetic
    x = generate_synthetic(3000, 64, 5)
    q = generate_synthetic(50, 64, 6)
    idx = BruteForceVectorIndex(64, metric)
    idx.add_batch([f"id{i}" for i in range(3000)], x)
    for i in range(0, 3000, 9):
        idx.delete(f"id{i}")
    idx.upsert("id5", x[7])
    idx.add("late", x[11])
    path = str(tmp_path / "flat")
    idx.snapshot(path)
    other = BruteForceVectorIndex(64, metric)
    other.add("junk", x[0])  # replaced by Load (Clear, :98)
    other.load(path)
    assert other.get_stats().count == idx.get_stats().count
    for opts in [None, SearchOptions(max_scans=500)]:
        a = idx.search_batch(q, 10, opts)
        b = other.search_batch(q, 10, opts)
        np.testing.assert_array_equal(a[1] >= 0, b[1] >= 0)
        # labels match through the ids (the shim's map travels with the image)
        for i in range(len(q)):
            ra = [r.id for r in idx.search(q[i], 10, opts)]
            rb = [r.id for r in other.search(q[i], 10, opts)]
            assert ra == rb
        assert np.array_equal(a[0].view(np.uint32), b[0].view(np.uint32))
    assert [i for i, _ in other.scan()] == [i for i, _ in idx.scan()]


@pytest.mark.parametrize("metric", [0, 1, 2])
def test_ivf_flat_round_trip(hiplib, tmp_path, metric):
    from pyrope_amd import IvfFlatVectorIndex, SearchOptions, generate_synthetic
    x = generate_synthetic(20000, 32, 7)
    q = generate_synthetic(200, 32, 8)
    idx = IvfFlatVectorIndex(32, metric, n_list=16)
    idx.add_batch([f"v{i}" for i in range(20000)], x)
    idx.build()
    for i in range(0, 20000, 13):  # removed from the lists
        idx.delete(f"v{i}")
    idx.add_batch([f"v{i}" for i in range(1, 400, 3)], x[2:401:3])  # buffer rows shadowing list rows
    idx.add("new", x[5])
    path = str(tmp_path / "ivf")
    idx.snapshot(path)
    other = IvfFlatVectorIndex(32, metric, n_list=16)
    other.load(path)
    assert other.get_stats().count == idx.get_stats().count
    np.testing.assert_array_equal(other.centroids_array(), idx.centroids_array())
    for opts in [SearchOptions(nprobe=4), SearchOptions(nprobe=16, max_scans=3000)]:
        _same(idx.search_batch(q, 10, opts), other.search_batch(q, 10, opts))
    other.build()  # and the loaded index rebuilds like the original
    idx.build()
    _same(idx.search_batch(q, 10, SearchOptions(nprobe=4)), other.search_batch(q, 10, SearchOptions(nprobe=4)))


def test_ivf_pq_round_trip(hiplib, tmp_path):
    from pyrope_amd import IvfPqVectorIndex, SearchOptions, generate_synthetic
    x = generate_synthetic(6000, 64, 9)
    q = generate_synthetic(100, 64, 10)
    idx = IvfPqVectorIndex(64, 0, m=8, k=64, n_list=8)
    idx.add_batch([f"p{i}" for i in range(6000)], x)
    idx.build()
    idx.add("p3", x[4])  # a buffer row hiding a list entry
    path = str(tmp_path / "pq")
    idx.snapshot(path)
    other = IvfPqVectorIndex(64, 0, m=8, k=64, n_list=8)
    other.load(path)
    cb1, codes1, off1, lab1, live1 = idx.pq_state()
    cb2, codes2, off2, lab2, live2 = other.pq_state()
    np.testing.assert_array_equal(cb1, cb2)
    np.testing.assert_array_equal(codes1, codes2)
    np.testing.assert_array_equal(lab1, lab2)
    np.testing.assert_array_equal(live1, live2)
    _same(idx.search_batch(q, 10, SearchOptions(nprobe=3)), other.search_batch(q, 10, SearchOptions(nprobe=3)))


def test_delta_manifest_round_trip(hiplib, tmp_path):  # DeltaVectorIndex.cs:160-212
    from pyrope_amd import VectorIndexRegistry, VectorMetric
    reg = VectorIndexRegistry()
    d = reg.create(8, VectorMetric.L2, "IVF_FLAT", {"nlist": 4})
    rng = np.random.default_rng(1)
    x = rng.random((300, 8), dtype=np.float32)
    for i in range(200):
        d.add(f"t{i}", x[i])
    d.build()  # compacts the head into the tail
    for i in range(200, 300):
        d.add(f"h{i}", x[i])  # stays in the head
    path = str(tmp_path / "delta")
    d.snapshot(path)
    assert open(path).read() == '{"Type": "Delta", "Head": ".head", "Tail": ".tail"}'
    for suffix in [".head", ".tail"]:
        assert os.path.exists(path + suffix) and not os.path.exists(path + suffix + ".tmp")
    e = reg.create(8, VectorMetric.L2, "IVF_FLAT", {"nlist": 4})
    e.load(path)
    assert e.get_stats().count == d.get_stats().count
    for i in range(0, 300, 7):
        assert [r.id for r in e.search(x[i], 5)] == [r.id for r in d.search(x[i], 5)]


@pytest.mark.parametrize("kind", ["flat", "ivf"])
def test_load_without_id_map_keeps_labels_unique(hiplib, tmp_path, kind):
    """an image loaded without the shim's .ids map (written by pyr_index_snapshot directly
    or by another client) exposes its rows as str(label) ids; a new id must get a label above every
    loaded one (no collision with row '0'), and deleting a loaded id must work."""
    from pyrope_amd import BruteForceVectorIndex, IvfFlatVectorIndex, VectorMetric, generate_synthetic
    mk = (lambda: BruteForceVectorIndex(16, VectorMetric.L2)) if kind == "flat" else \
        (lambda: IvfFlatVectorIndex(16, VectorMetric.L2, n_list=4))
    x = generate_synthetic(300, 16, 3)
    idx = mk()
    idx.add_labels(np.arange(300, dtype=np.int64), x)
    if kind == "ivf":
        idx.build()
        idx.add_labels(np.array([300, 301], np.int64), x[:2] + 1.0)  # buffer rows after the build
    path = str(tmp_path / "img")
    idx.snapshot(path)
    os.remove(path + ".ids")
    loaded = mk()
    loaded.load(path)
    n_rows = 300 if kind == "flat" else 302
    assert loaded._next_label == n_rows
    loaded.add("fresh", np.full(16, 7.0, np.float32))  # FLAT would raise on a reused label 0
    res = loaded.search(np.full(16, 7.0, np.float32), 1)
    assert res[0].id == "fresh"
    assert loaded.delete("0")
    assert "0" not in [r.id for r in loaded.search(x[0], 5)]


def test_stale_id_map_is_ignored(hiplib, tmp_path):
    """the .ids map records the nonce of the image it belongs to; an image replaced
    without its map (a crash between the two renames) loads with str(label) ids and a warning
    instead of another image's ids -- also when both images have the same size."""
    from pyrope_amd import BruteForceVectorIndex, VectorMetric
    a = BruteForceVectorIndex(4, VectorMetric.L2)
    a.add("alpha", [1, 0, 0, 0])
    a.add("beta", [0, 1, 0, 0])
    path = str(tmp_path / "img")
    a.snapshot(path)
    ids_a = open(path + ".ids").read()
    b = BruteForceVectorIndex(4, VectorMetric.L2)
    b.add("gamma", [0, 0, 1, 0])
    b.add("delta", [0, 0, 0, 1])
    b.add("eps", [1, 1, 0, 0])
    b.snapshot(path)
    open(path + ".ids", "w").write(ids_a)  # the previous snapshot's map next to the new image
    c = BruteForceVectorIndex(4, VectorMetric.L2)
    with pytest.warns(RuntimeWarning, match="nonce"):
        c.load(path)
    assert c.search([0, 0, 1, 0], 1)[0].id == "0"
    assert c._next_label == 3
    # same content, same size: the second snapshot's image still rejects the first one's map
    b.snapshot(path)
    ids_b = open(path + ".ids").read()
    b.snapshot(path)
    assert os.path.getsize(path) > 0
    open(path + ".ids", "w").write(ids_b)
    d = BruteForceVectorIndex(4, VectorMetric.L2)
    with pytest.warns(RuntimeWarning, match="nonce"):
        d.load(path)
    assert d.search([0, 0, 1, 0], 1)[0].id == "0"


def _strip_nonce(path):
    """Drop the trailing T_NONCE section (tag 13, 16 bytes: persist.h) and fix the header's section count."""
    b = bytearray(open(path, "rb").read())
    tag, _, n = struct.unpack_from("<IIQ", b, len(b) - 32)
    assert (tag, n) == (13, 16)
    del b[len(b) - 32:]
    nsec = struct.unpack_from("<I", b, 24)[0]
    struct.pack_into("<I", b, 24, nsec - 1)
    st = os.stat(path)
    open(path, "wb").write(bytes(b))
    os.utime(path, ns=(st.st_atime_ns, st.st_mtime_ns + 1))


def test_pre_nonce_snapshot_keeps_its_ids(hiplib, tmp_path):
    """a snapshot written before images carried a nonce (round 3: no T_NONCE section, an .ids map
    with 'image': [size, mtime_ns] and no 'image_nonce') still loads with its string ids; the same legacy
    map next to a newer image (which has a nonce) or a changed image is rejected."""
    import json
    from pyrope_amd import BruteForceVectorIndex, VectorMetric
    a = BruteForceVectorIndex(4, VectorMetric.L2)
    a.add("alpha", [1, 0, 0, 0])
    a.add("beta", [0, 1, 0, 0])
    path = str(tmp_path / "old")
    a.snapshot(path)
    _strip_nonce(path)  # the image as round 3 wrote them: no T_NONCE section
    m = json.load(open(path + ".ids"))
    st = os.stat(path)
    legacy = {"next": m["next"], "image": [st.st_size, st.st_mtime_ns], "ids": m["ids"]}
    json.dump(legacy, open(path + ".ids", "w"))
    c = BruteForceVectorIndex(4, VectorMetric.L2)
    c.load(path)
    assert c.search([0, 1, 0, 0], 1)[0].id == "beta"
    # the legacy map beside an image with a nonce: rejected
    a.snapshot(path)
    json.dump(legacy, open(path + ".ids", "w"))
    d = BruteForceVectorIndex(4, VectorMetric.L2)
    with pytest.warns(RuntimeWarning, match="nonce"):
        d.load(path)
    assert d.search([0, 1, 0, 0], 1)[0].id == "1"


def test_corrupt_images_raise_format_errors(hiplib, tmp_path):
    """centroids that are not whole rows, and section sizes running past the end of the
    file (including sizes that would wrap the offset), are rejected as malformed images."""
    from pyrope_amd import IvfFlatVectorIndex
    from pyrope_amd._lib import JsonException
    p1 = str(tmp_path / "cents")
    _image(p1, 1, 4, 0, [(1, b"\1"), (2, np.zeros(6, np.float32).tobytes())])  # T_CENTS: 1.5 rows
    with pytest.raises(JsonException):
        IvfFlatVectorIndex(4, 0).load(p1)
    p2 = str(tmp_path / "wrap")
    with open(p2, "wb") as f:
        f.write(b"PYRIDX01" + struct.pack("<iiiiI", 1, 1, 4, 0, 2))
        f.write(struct.pack("<IIQ", 6, 0, 2 ** 64 - 8))  # wraps off back to the start
        f.write(struct.pack("<IIQ", 1, 0, 1) + b"\1" + b"\0" * 7)
    with pytest.raises(JsonException):
        IvfFlatVectorIndex(4, 0).load(p2)
