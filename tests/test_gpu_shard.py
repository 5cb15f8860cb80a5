"""List-sharded IVF_FLAT on the device (include/pyrope_ann.h "List-sharded multi-GPU"; shard.hip): W shard
indexes on one GPU, each holding WHOLE lists (dist.list_owners) plus the replicated list samples, driven
through the step's phases with the collectives done as tensor copies (the orchestration itself is tested
on gloo ranks in tests/test_dist_lists.py).  The answers must equal the unsharded index's bit for bit,
ids and scores, with the certificates as they fall and with every certificate forced to fail (every query
then comes back through the exact re-run).  Reference loop split across ranks: IvfFlatVectorIndex.cs:198-218.
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
    return idx


def _step(idx, q, nq, k, P, opts, fcap):
    """The ListShardedIvf phases for W ranks in one process; returns the homes' answers and failures."""
    import torch

    from pyrope_amd.dist import DeviceShardEngine
    W = len(idx)
    Q = nq * W
    rb = 16 * (k + 1)
    eng = [DeviceShardEngine(ix, k, opts) for ix in idx]
    plans = [torch.empty((nq, P + 1), dtype=torch.int32, device="cuda") for _ in range(W)]
    for r in range(W):
        assert eng[r].prepare(q[r * nq:(r + 1) * nq], plans[r]) == P
    plan_all = torch.cat(plans)
    recs = [torch.empty((Q, rb), dtype=torch.uint8, device="cuda") for _ in range(W)]
    for r in range(W):
        eng[r].search(q, plan_all, P, recs[r])
    out_s = torch.empty((Q, k), dtype=torch.float32, device="cuda")
    out_l = torch.empty((Q, k), dtype=torch.int64, device="cuda")
    fails = torch.zeros((W, 1 + fcap), dtype=torch.int32, device="cuda")
    for h in range(W):
        rh = torch.stack([recs[s][h * nq:(h + 1) * nq] for s in range(W)])  # the all_to_all's output at h
        eng[h].merge(rh, out_s[h * nq:(h + 1) * nq], out_l[h * nq:(h + 1) * nq], fails[h])
    rrec = [torch.zeros((W * fcap, rb), dtype=torch.uint8, device="cuda") for _ in range(W)]
    for r in range(W):
        eng[r].rerun(q, plan_all, P, fails, nq, rrec[r])
    for h in range(W):
        rh = torch.stack([rrec[s][h * fcap:(h + 1) * fcap] for s in range(W)])
        eng[h].merge_rerun(rh, fails[h], out_s[h * nq:(h + 1) * nq], out_l[h * nq:(h + 1) * nq])
    torch.cuda.synchronize()
    return out_s.cpu().numpy(), out_l.cpu().numpy(), fails[:, 0].cpu().numpy()


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("metric", [0, 1])
@pytest.mark.parametrize("force_fail", [False, True])
def test_list_sharded_equals_unsharded(hiplib, world, metric, force_fail):
    import torch

    from pyrope_amd import IvfFlatVectorIndex, SearchOptions, generate_synthetic, kmeans_train
    n, d, nl, P, k, nq = 40_000, 128, 64, 8, 10, 150
    data = generate_synthetic(n, d, 42)
    cents = kmeans_train(data, nl, metric, 8, 42)
    qh = generate_synthetic(nq * world, d, 1337)
    opts = SearchOptions(nprobe=P)
    full = IvfFlatVectorIndex(d, metric, n_list=nl)
    full.set_centroids(cents)
    full.add_labels(np.arange(n, dtype=np.int64), data, track_ids=False)
    full.build()
    ref_s, ref_l, _ = full.search_batch(qh, k, opts)
    idx = _shards(data, cents, world, metric)
    q = torch.from_numpy(qh).cuda()
    env = {"PYR_FILTER_CERR": "1e15"} if force_fail else {}
    with _env(**env):
        s, lab, nfail = _step(idx, q, nq, k, P, opts, fcap=nq)
    np.testing.assert_array_equal(lab, ref_l)
    assert np.array_equal(s.view(np.uint32), ref_s.view(np.uint32))
    if force_fail:
        assert (nfail == nq).all()   # every certificate failed: all answers came from the exact re-run
    else:
        assert nfail.sum() <= world * 2


def test_list_sharded_exact_ties_across_lists(hiplib):
    """Rows at exactly equal distance from a query in different lists (often on different ranks): on a
    grid of multiples of 2^-6 the reflection 2q - x of a row x about q is exact, so |q - x|^2 ties bit for
    bit.  The merged order must be the unsharded index's storage order, (list asc, label asc)."""
    import torch

    from pyrope_amd import IvfFlatVectorIndex, SearchOptions, generate_synthetic, kmeans_train
    n, d, nl, P, k, nq, world = 20_000, 64, 32, 32, 20, 64, 2
    data = np.round(generate_synthetic(n, d, 7) * 64) / 64
    cents = kmeans_train(data, nl, 0, 8, 42)
    qh = (np.round(generate_synthetic(nq * world, d, 9) * 64) / 64).astype(np.float32)
    refl = []
    for q in qh[: nq]:  # the 6 nearest rows of half of the queries, reflected about the query
        near = np.argsort(((data - q) ** 2).sum(1))[:6]
        refl.append(2 * q - data[near])
    data = np.concatenate([data] + refl).astype(np.float32)
    n = len(data)
    opts = SearchOptions(nprobe=P)
    full = IvfFlatVectorIndex(d, 0, n_list=nl)
    full.set_centroids(cents)
    full.add_labels(np.arange(n, dtype=np.int64), data, track_ids=False)
    full.build()
    ref_s, ref_l, _ = full.search_batch(qh, k, opts)
    # the construction does produce exact ties inside the top-k
    assert sum(len(set(r.tolist())) < k for r in ref_s[:nq]) > nq // 2
    idx = _shards(data, cents, world)
    s, lab, _ = _step(idx, torch.from_numpy(qh).cuda(), nq, k, P, opts, fcap=nq)
    np.testing.assert_array_equal(lab, ref_l)
    assert np.array_equal(s.view(np.uint32), ref_s.view(np.uint32))
