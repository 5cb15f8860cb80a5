"""List-sharded IVF_FLAT on the device (include/pyrope_ann.h "List-sharded multi-GPU"; shard.hip): W shard
indexes on one GPU, each holding WHOLE lists (dist.list_owners) plus the replicated list samples, driven by the
bench's own orchestration (dist.ListShardedIvf) with the collectives done as device copies between the ranks'
buffers (dist.LocalShardGroup; the collectives themselves run on gloo ranks in tests/test_dist_lists.py).  The
answers must equal the unsharded index's bit for bit, ids and scores, with the certificates as they fall, with
every certificate forced to fail (every query then comes back through the exact re-run), with more failures
than one re-run round carries (further rounds), under a MaxScans budget, and at the M8 coarse shape (world 8,
nlist 8192, nprobe 32) against the oracle too.  Reference loop split across ranks: IvfFlatVectorIndex.cs:198-218
(MaxScans: :152-156, :202-212).
"""
import ctypes as C
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


def _shards(data, cents, world, metric=0):
    from pyrope_amd import IvfFlatVectorIndex, assign
    from pyrope_amd.dist import SAMPLE_ROWS, list_owners
    a = assign(cents, data, metric)
    glen = np.bincount(a, minlength=len(cents))
    owner = list_owners(glen, world)
    order = np.argsort(a, kind="stable")  # list-major, label order inside a list
    off = np.concatenate([[0], np.cumsum(glen)])
    counts = np.minimum(glen, SAMPLE_ROWS)
    srows = np.concatenate([data[order[off[l]:off[l] + counts[l]]] for l in range(len(cents))])
    idx = []
    for r in range(world):
        ix = IvfFlatVectorIndex(data.shape[1], metric, n_list=len(cents))
        ix.set_centroids(cents)
        labs = np.nonzero(owner[a] == r)[0].astype(np.int64)  # label order
        ix.add_labels(labs, data[labs], track_ids=False)
        ix.build()
        ix.set_list_samples(srows, counts, glen)
        idx.append(ix)
    return idx, owner, a


def _run(idx, q, nq, k, P, opts, fcap, steps=1):
    """dist.ListShardedIvf for W ranks in one process -> (scores [W nq, k], labels, per-rank step objects)."""
    import torch

    from pyrope_amd.dist import DeviceShardEngine, ListShardedIvf, LocalShardGroup
    W = len(idx)
    steps_ = [ListShardedIvf(DeviceShardEngine(ix, k, opts), None, nq, k, P, r, W, device="cuda", fcap=fcap)
              for r, ix in enumerate(idx)]
    grp = LocalShardGroup(steps_)
    for _ in range(steps):
        out = grp(q)
    torch.cuda.synchronize()
    s = torch.cat([o[0] for o in out]).cpu().numpy()
    lab = torch.cat([o[1] for o in out]).cpu().numpy()
    return s, lab, steps_


def _unsharded(data, cents, metric, qh, k, opts):
    from pyrope_amd import IvfFlatVectorIndex
    full = IvfFlatVectorIndex(data.shape[1], metric, n_list=len(cents))
    full.set_centroids(cents)
    full.add_labels(np.arange(len(data), dtype=np.int64), data, track_ids=False)
    full.build()
    ref_s, ref_l, _ = full.search_batch(qh, k, opts)
    return full, ref_s, ref_l


def _same(s, lab, ref_s, ref_l):
    np.testing.assert_array_equal(lab, ref_l)
    assert np.array_equal(s.view(np.uint32), ref_s.view(np.uint32))


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("metric", [0, 1])
@pytest.mark.parametrize("force_fail", [False, True])
def test_list_sharded_equals_unsharded(hiplib, world, metric, force_fail):
    import torch

    from pyrope_amd import SearchOptions, generate_synthetic, kmeans_train
    n, d, nl, P, k, nq = 40_000, 128, 64, 8, 10, 150
    data = generate_synthetic(n, d, 42)
    cents = kmeans_train(data, nl, metric, 8, 42)
    qh = generate_synthetic(nq * world, d, 1337)
    opts = SearchOptions(nprobe=P)
    _, ref_s, ref_l = _unsharded(data, cents, metric, qh, k, opts)
    idx, _, _ = _shards(data, cents, world, metric)
    q = torch.from_numpy(qh).cuda()
    env = {"PYR_FILTER_CERR": "1e15"} if force_fail else {}
    with _env(**env):
        s, lab, st = _run(idx, q, nq, k, P, opts, fcap=nq)
    _same(s, lab, ref_s, ref_l)
    if force_fail:
        assert st[0].stats["max_failures"] == nq   # every certificate failed: all answers from the exact re-run
    else:
        assert st[0].stats["max_failures"] <= 2


@pytest.mark.parametrize("fcap", [1, 16, 64])
def test_list_sharded_more_failures_than_fcap(hiplib, fcap):
    """a home with more certificate failures than one re-run round carries.  Every certificate
    is forced to fail (150 per home), so the step runs ceil(150 / fcap) re-run rounds; twice in a row (the
    second step reuses every buffer, the rounds' fail lists included).  Must equal the unsharded index."""
    import torch

    from pyrope_amd import SearchOptions, generate_synthetic, kmeans_train
    n, d, nl, P, k, nq, world = 30_000, 64, 48, 6, 10, 150, 3
    data = generate_synthetic(n, d, 5)
    cents = kmeans_train(data, nl, 0, 6, 42)
    qh = generate_synthetic(nq * world, d, 77)
    opts = SearchOptions(nprobe=P)
    _, ref_s, ref_l = _unsharded(data, cents, 0, qh, k, opts)
    idx, _, _ = _shards(data, cents, world)
    with _env(PYR_FILTER_CERR="1e15"):
        s, lab, st = _run(idx, torch.from_numpy(qh).cuda(), nq, k, P, opts, fcap=fcap, steps=2)
    _same(s, lab, ref_s, ref_l)
    assert st[0].stats == {"max_failures": nq, "extra_rounds": (nq - 1) // fcap}


@pytest.mark.parametrize("metric", [0, 1])
@pytest.mark.parametrize("max_scans", [0, 1, 700, 3000, 12000])
def test_list_sharded_max_scans(hiplib, oracle, metric, max_scans):
    """SearchOptions.MaxScans (IvfFlatVectorIndex.cs:202-212) on the list-sharded step: the home runs the budget
    down the probe order over every rank's lists, the owners stop where it ran out.  Equal to the unsharded
    index under the same budget (itself oracle-identical, tests/test_gpu_maxscans.py) and to the oracle on a
    sample of queries; certificates as they fall and all forced to fail (the re-run honours the budget)."""
    import torch

    from pyrope_amd import SearchOptions, generate_synthetic, kmeans_train
    n, d, nl, P, k, nq, world = 40_000, 128, 64, 8, 10, 120, 3
    data = generate_synthetic(n, d, 11)
    cents = kmeans_train(data, nl, metric, 6, 42)
    qh = generate_synthetic(nq * world, d, 12)
    opts = SearchOptions(nprobe=P, max_scans=max_scans)
    full, ref_s, ref_l = _unsharded(data, cents, metric, qh, k, opts)
    idx, _, _ = _shards(data, cents, world, metric)
    q = torch.from_numpy(qh).cuda()
    s, lab, st = _run(idx, q, nq, k, P, opts, fcap=32)
    _same(s, lab, ref_s, ref_l)
    assert st[0].budget and st[0].plan_all.shape[1] == 2 * P + 1
    with _env(PYR_FILTER_CERR="1e15"):
        s2, lab2, _ = _run(idx, q, nq, k, P, opts, fcap=32)
    _same(s2, lab2, ref_s, ref_l)
    off, labels, live = full.ivf_layout()
    rows = data[labels]
    for i in range(0, nq * world, 37):
        os_, ok = oracle.ivf_search(qh[i], k, full.centroids_array(), rows, off, live, metric=metric, nprobe=P,
                                    max_scans=max_scans)
        c = len(os_)
        np.testing.assert_array_equal(lab[i, :c], labels[ok])
        assert np.array_equal(s[i, :c].view(np.uint32), os_.view(np.uint32))
        assert (lab[i, c:] == -1).all()


def test_list_sharded_max_scans_refused_after_deletes(hiplib):
    """A Delete on a rank changes its lists' live lengths, which the other ranks' homes used to run the budget
    down: a budgeted step must fail loudly (PYR_E_STATE) until the samples are set again; unbudgeted searches
    stay correct."""
    import torch

    from pyrope_amd import SearchOptions, _lib, generate_synthetic, kmeans_train
    from pyrope_amd._lib import InvalidOperationException
    n, d, nl, P, k, nq, world = 20_000, 64, 32, 6, 10, 64, 2
    data = generate_synthetic(n, d, 3)
    cents = kmeans_train(data, nl, 0, 5, 42)
    idx, owner, a = _shards(data, cents, world)
    gone = np.nonzero(owner[a] == 1)[0][:5].astype(np.int64)
    L = _lib.load()
    _lib.check(L.pyr_index_remove(idx[1]._h, gone.ctypes.data_as(C.POINTER(C.c_int64)), len(gone), None))
    q = torch.from_numpy(generate_synthetic(nq * world, d, 4)).cuda()
    with pytest.raises(InvalidOperationException, match="MaxScans"):
        _run(idx, q, nq, k, P, SearchOptions(nprobe=P, max_scans=5000), fcap=16)
    keep = np.setdiff1d(np.arange(n), gone)
    _, ref_s, ref_l = _unsharded(data[keep], cents, 0, q.cpu().numpy(), k, SearchOptions(nprobe=P))
    s, lab, _ = _run(idx, q, nq, k, P, SearchOptions(nprobe=P), fcap=16)
    np.testing.assert_array_equal(lab, np.where(ref_l >= 0, keep[np.maximum(ref_l, 0)], -1))
    assert np.array_equal(s.view(np.uint32), ref_s.view(np.uint32))


def test_list_sharded_world8_m8_coarse_shape(hiplib, oracle):
    """the M8 configuration's partition -- 8 ranks, nlist 8192, nprobe 32 (at small N) -- against
    the unsharded index (every query) and the oracle (a sample)."""
    import torch

    from pyrope_amd import SearchOptions, generate_synthetic, kmeans_train
    n, d, nl, P, k, nq, world = 120_000, 128, 8192, 32, 10, 64, 8
    data = generate_synthetic(n, d, 21)
    cents = kmeans_train(data, nl, 0, 3, 42)
    qh = generate_synthetic(nq * world, d, 22)
    opts = SearchOptions(nprobe=P)
    full, ref_s, ref_l = _unsharded(data, cents, 0, qh, k, opts)
    idx, owner, _ = _shards(data, cents, world)
    assert len(np.unique(owner)) == world
    s, lab, st = _run(idx, torch.from_numpy(qh).cuda(), nq, k, P, opts, fcap=256)
    _same(s, lab, ref_s, ref_l)
    off, labels, live = full.ivf_layout()
    rows = data[labels]
    for i in range(0, nq * world, 41):
        os_, ok = oracle.ivf_search(qh[i], k, full.centroids_array(), rows, off, live, nprobe=P)
        np.testing.assert_array_equal(lab[i], labels[ok])
        assert np.array_equal(s[i].view(np.uint32), os_.view(np.uint32))


def test_list_sharded_exact_ties_across_lists(hiplib):
    """Rows at exactly equal distance from a query in different lists (often on different ranks): on a
    grid of multiples of 2^-6 the reflection 2q - x of a row x about q is exact, so |q - x|^2 ties bit for
    bit.  The merged order must be the unsharded index's storage order, (list asc, label asc)."""
    import torch

    from pyrope_amd import SearchOptions, generate_synthetic, kmeans_train
    n, d, nl, P, k, nq, world = 20_000, 64, 32, 32, 20, 64, 2
    data = np.round(generate_synthetic(n, d, 7) * 64) / 64
    cents = kmeans_train(data, nl, 0, 8, 42)
    qh = (np.round(generate_synthetic(nq * world, d, 9) * 64) / 64).astype(np.float32)
    refl = []
    for q in qh[: nq]:  # the 6 nearest rows of half of the queries, reflected about the query
        near = np.argsort(((data - q) ** 2).sum(1))[:6]
        refl.append(2 * q - data[near])
    data = np.concatenate([data] + refl).astype(np.float32)
    opts = SearchOptions(nprobe=P)
    _, ref_s, ref_l = _unsharded(data, cents, 0, qh, k, opts)
    # the construction does produce exact ties inside the top-k
    assert sum(len(set(r.tolist())) < k for r in ref_s[:nq]) > nq // 2
    idx, _, _ = _shards(data, cents, world)
    s, lab, _ = _run(idx, torch.from_numpy(qh).cuda(), nq, k, P, opts, fcap=nq)
    _same(s, lab, ref_s, ref_l)


def test_list_sharded_phase_graphs_capture_and_replay(hiplib):
    """ListShardedIvf.capture (bench.py's N > 1 step): the five device phases captured into hipGraphs after a step
    that had no failures (so the re-run's workspaces are sized outside the capture), replayed twice, equal to the
    unsharded index; a rank of one (dist.Comm(1): the collectives as copies)."""
    import torch

    from pyrope_amd import SearchOptions, generate_synthetic, kmeans_train
    from pyrope_amd.dist import Comm, DeviceShardEngine, ListShardedIvf
    n, d, nl, P, k, nq = 30_000, 128, 48, 6, 10, 200
    data = generate_synthetic(n, d, 31)
    cents = kmeans_train(data, nl, 0, 6, 42)
    qh = generate_synthetic(nq, d, 32)
    opts = SearchOptions(nprobe=P)
    _, ref_s, ref_l = _unsharded(data, cents, 0, qh, k, opts)
    idx, _, _ = _shards(data, cents, 1)
    q = torch.from_numpy(qh).cuda()
    step = ListShardedIvf(DeviceShardEngine(idx[0], k, opts), Comm(1), nq, k, P, 0, 1, device="cuda")
    step(q)
    torch.cuda.synchronize()
    assert step.stats["max_failures"] == 0
    step.capture(q)
    for _ in range(2):
        step.out_s.fill_(0)
        step.out_l.fill_(-7)
        s, lab = step(q)
        torch.cuda.synchronize()
        _same(s.cpu().numpy(), lab.cpu().numpy(), ref_s, ref_l)


def test_list_sharded_repeatable_large_items(hiplib):
    """Full 512-query items with many emitted rows per item on every rank (long lists, a low fixed sample rank):
    three steps in a row, each equal to the unsharded index.  Round 6's flush / next-prologue race (fixed,
    profiles/r6_race/) showed at this kind of shape as answers that changed from step to step."""
    import torch

    from pyrope_amd import SearchOptions, generate_synthetic, kmeans_train
    n, d, nl, P, k, nq, world = 200_000, 64, 32, 8, 10, 2000, 4
    data = generate_synthetic(n, d, 31)
    cents = kmeans_train(data, nl, 0, 4, 42)
    qh = generate_synthetic(nq * world, d, 32)
    opts = SearchOptions(nprobe=P)
    _, ref_s, ref_l = _unsharded(data, cents, 0, qh, k, opts)
    idx, _, _ = _shards(data, cents, world)
    q = torch.from_numpy(qh).cuda()
    with _env(PYR_STREAM_RANK=48):
        for _ in range(3):
            s, lab, _ = _run(idx, q, nq, k, P, opts, fcap=256)
            _same(s, lab, ref_s, ref_l)
