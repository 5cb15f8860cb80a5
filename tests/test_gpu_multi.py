"""The multi-GPU index behind the C ABI (pyr_index_desc.device_mask / shards; csrc/multi.cpp).

One pyr_index whose lists are dealt whole to W shard indexes and searched by the list-sharded step inside the
library (the reference serves an index from one process, Extensions/VectorCommandSet.cs:457-459, created by one
constructor call, Services/VectorIndexRegistry.cs:81-113).  On a one-GPU box: W shards on device 0 with the
collectives as device copies, and one shard over RCCL (a one-rank communicator: the RCCL calls themselves).
Every answer must equal the single-GPU index's, ids and score bits, through the same IVectorIndex calls:
Add / Build / Search (host and device buffers) / Delete / Upsert / rebuild / Snapshot / Load, MaxScans,
forced certificate failures and more failures than one re-run round, batches not divisible by W, and the
paths the step does not take (Cosine, k > 60, a non-empty buffer) answered by the first-device index.
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


def _pair(data, metric, nl, shards, mask=1, labels=None):
    from pyrope_amd import IvfFlatVectorIndex
    labels = np.arange(len(data), dtype=np.int64) if labels is None else labels
    one = IvfFlatVectorIndex(data.shape[1], metric, n_list=nl)
    multi = IvfFlatVectorIndex(data.shape[1], metric, n_list=nl, device_mask=mask, shards=shards)
    for ix in (one, multi):
        ix.add_labels(labels, data, track_ids=False)
        ix.build()
    return one, multi


def _same(a, b):
    (s1, l1, c1), (s2, l2, c2) = a, b
    np.testing.assert_array_equal(l2, l1)
    assert np.array_equal(s2.view(np.uint32), s1.view(np.uint32))
    np.testing.assert_array_equal(c2, c1)


@pytest.mark.parametrize("shards", [2, 3, 4])
@pytest.mark.parametrize("metric", [0, 1])
def test_multi_index_equals_single(hiplib, shards, metric):
    from pyrope_amd import SearchOptions, generate_synthetic
    data = generate_synthetic(30_000, 128, 42)
    one, multi = _pair(data, metric, 48, shards)
    info = multi.shard_info()
    assert info["shards"] == shards
    q = generate_synthetic(301, 128, 1337)  # 301: not a multiple of the shard count (padded home batches)
    for opts in (SearchOptions(nprobe=6), SearchOptions(nprobe=48), SearchOptions(nprobe=6, max_scans=900)):
        _same(one.search_batch(q, 10, opts), multi.search_batch(q, 10, opts))
    info = multi.shard_info()
    assert info["xport"] == "copy" and info["sharded_searches"] == 3 and info["staged_searches"] == 0


def test_one_device_mask_is_the_single_gpu_index(hiplib):
    from pyrope_amd import SearchOptions, generate_synthetic
    data = generate_synthetic(20_000, 64, 5)
    one, multi = _pair(data, 0, 32, 0, mask=1)
    assert multi.shard_info()["shards"] == 1
    q = generate_synthetic(100, 64, 6)
    _same(one.search_batch(q, 10, SearchOptions(nprobe=5)), multi.search_batch(q, 10, SearchOptions(nprobe=5)))


def test_one_shard_over_rccl(hiplib):
    """shards = 1 on a one-device mask: the list-sharded step with a one-rank RCCL communicator
    (ncclCommInitAll, grouped broadcast / all_gather / all_to_all on the shard stream)."""
    from pyrope_amd import SearchOptions, generate_synthetic
    data = generate_synthetic(20_000, 128, 8)
    one = _pair(data, 0, 32, 0)[0]
    from pyrope_amd import IvfFlatVectorIndex
    multi = IvfFlatVectorIndex(128, 0, n_list=32, device_mask=1, shards=1)
    with _env(PYR_SHARD_XPORT="rccl"):
        multi.add_labels(np.arange(len(data), dtype=np.int64), data, track_ids=False)
        multi.build()
        q = generate_synthetic(200, 128, 9)
        with _env(PYR_FILTER_CERR="1e15"):  # every certificate fails: the re-run's collectives too
            _same(one.search_batch(q, 10, SearchOptions(nprobe=4)), multi.search_batch(q, 10, SearchOptions(nprobe=4)))
        _same(one.search_batch(q, 10, SearchOptions(nprobe=4)), multi.search_batch(q, 10, SearchOptions(nprobe=4)))
    info = multi.shard_info()
    assert info["xport"] == "rccl" and info["sharded_searches"] == 2


def test_multi_index_failures_past_fcap(hiplib):
    """Every certificate forced to fail with a 16-failure re-run round: 10 rounds per home per step."""
    from pyrope_amd import IvfFlatVectorIndex, SearchOptions, generate_synthetic
    data = generate_synthetic(25_000, 64, 10)
    one = _pair(data, 0, 40, 0)[0]
    with _env(PYR_SHARD_FCAP=16):
        multi = IvfFlatVectorIndex(64, 0, n_list=40, device_mask=1, shards=3)
    multi.add_labels(np.arange(len(data), dtype=np.int64), data, track_ids=False)
    multi.build()
    q = generate_synthetic(480, 64, 11)
    with _env(PYR_FILTER_CERR="1e15"):
        got = multi.search_batch(q, 10, SearchOptions(nprobe=5, max_scans=3000))
    _same(one.search_batch(q, 10, SearchOptions(nprobe=5, max_scans=3000)), got)
    info = multi.shard_info()
    assert info["last_max_failures"] == 160 and info["last_extra_rounds"] == 9


def test_multi_index_device_search_and_graphless_stream(hiplib):
    import torch

    from pyrope_amd import SearchOptions, generate_synthetic
    data = generate_synthetic(30_000, 128, 12)
    one, multi = _pair(data, 0, 64, 4)
    qh = generate_synthetic(1000, 128, 13)
    q = torch.from_numpy(qh).cuda()
    k = 20
    s = torch.empty((1000, k), dtype=torch.float32, device="cuda")
    lab = torch.empty((1000, k), dtype=torch.int64, device="cuda")
    cnt = torch.empty((1000,), dtype=torch.int32, device="cuda")
    st = torch.cuda.Stream()
    with torch.cuda.stream(st):
        multi.search_device(q.data_ptr(), 1000, k, s.data_ptr(), lab.data_ptr(), cnt.data_ptr(), st.cuda_stream,
                            SearchOptions(nprobe=8))
    st.synchronize()
    _same(one.search_batch(qh, k, SearchOptions(nprobe=8)), (s.cpu().numpy(), lab.cpu().numpy(), cnt.cpu().numpy()))


def test_multi_index_writes_rebuild_and_stage_paths(hiplib):
    """The IVectorIndex write path on the multi-GPU index, step by step beside the single-GPU index:
    Delete after Build (the shards drop the rows; MaxScans accounting follows), Upsert of a built row and Add
    of new rows (a non-empty buffer: answered by the first-device index), rebuild (dealt again), Cosine-free
    k > 60 (the first-device index), Snapshot / Load."""
    import ctypes as C

    from pyrope_amd import SearchOptions, generate_synthetic
    from pyrope_amd._lib import check
    data = generate_synthetic(24_000, 64, 14)
    one, multi = _pair(data, 0, 32, 3)
    q = generate_synthetic(150, 64, 15)
    opts = SearchOptions(nprobe=6, max_scans=2500)
    gone = np.arange(0, 24_000, 7, dtype=np.int64)
    for ix in (one, multi):
        check(ix._L.pyr_index_remove(ix._h, gone.ctypes.data_as(C.POINTER(C.c_int64)), len(gone), None))
    _same(one.search_batch(q, 10, opts), multi.search_batch(q, 10, opts))
    _same(one.search_batch(q, 10), multi.search_batch(q, 10))
    before = multi.shard_info()["sharded_searches"]
    new = generate_synthetic(500, 64, 16)
    labs = np.concatenate([np.arange(1, 400, 2), np.arange(30_000, 30_300)]).astype(np.int64)
    for ix in (one, multi):
        ix.add_labels(labs, new, track_ids=False)
    _same(one.search_batch(q, 10, opts), multi.search_batch(q, 10, opts))  # buffer rows: the stage
    assert multi.shard_info()["sharded_searches"] == before
    for ix in (one, multi):
        ix.build()
    _same(one.search_batch(q, 10, opts), multi.search_batch(q, 10, opts))
    assert multi.shard_info()["sharded_searches"] == before + 1
    _same(one.search_batch(q, 100, SearchOptions(nprobe=6)), multi.search_batch(q, 100, SearchOptions(nprobe=6)))


def test_multi_index_snapshot_load(hiplib, tmp_path):
    from pyrope_amd import IvfFlatVectorIndex, SearchOptions, generate_synthetic
    data = generate_synthetic(20_000, 64, 17)
    one, multi = _pair(data, 1, 32, 2)
    p = str(tmp_path / "m.idx")
    multi.snapshot(p)
    back = IvfFlatVectorIndex(64, 1, n_list=32, device_mask=1, shards=3)
    back.load(p)
    q = generate_synthetic(120, 64, 18)
    _same(one.search_batch(q, 10, SearchOptions(nprobe=7)), back.search_batch(q, 10, SearchOptions(nprobe=7)))
    assert back.shard_info()["sharded_searches"] == 1


def test_multi_index_cosine_on_the_first_device(hiplib):
    from pyrope_amd import SearchOptions, generate_synthetic
    data = generate_synthetic(12_000, 64, 19) - 0.5
    one, multi = _pair(data.astype(np.float32), 2, 24, 2)
    q = (generate_synthetic(80, 64, 20) - 0.5).astype(np.float32)
    _same(one.search_batch(q, 10, SearchOptions(nprobe=4)), multi.search_batch(q, 10, SearchOptions(nprobe=4)))
    assert multi.shard_info()["staged_searches"] >= 1


def test_multi_index_small_batches(hiplib):
    """Fewer queries than shards (empty home slices) and a single query."""
    from pyrope_amd import SearchOptions, generate_synthetic
    data = generate_synthetic(16_000, 128, 21)
    one, multi = _pair(data, 0, 32, 4)
    for nq in (1, 2, 3, 5):
        q = generate_synthetic(nq, 128, 22 + nq)
        _same(one.search_batch(q, 10, SearchOptions(nprobe=5)), multi.search_batch(q, 10, SearchOptions(nprobe=5)))


def test_multi_index_rejects_other_kinds(hiplib):
    from pyrope_amd import BruteForceVectorIndex, IvfPqVectorIndex
    with pytest.raises(Exception, match="IVF_FLAT"):
        BruteForceVectorIndex(64, 0, device_mask=1, shards=2)
    with pytest.raises(Exception, match="IVF_FLAT"):
        IvfPqVectorIndex(64, 0, m=8, k=256, n_list=16, device_mask=1, shards=2)
