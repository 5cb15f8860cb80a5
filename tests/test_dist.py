"""Multi-GPU sharding (pyrope_amd/dist.py; SURVEY.md 8(e) option ii, rows within lists).

Rank r holds the generator blocks b with b % world == r and builds its lists with the shared
coarse quantizer, so the union of the ranks' probed rows is exactly the unsharded index's probed
rows, each scored with the same arithmetic.  One all_gather of the per-rank top-k partials + a merge by
(score desc, label asc) must then give the unsharded result (ties between equal scores in
different lists aside, which random fp32 data does not produce).

CPU tests run the orchestration with gloo at world size 2 (the per-rank scan is the oracle, as
the GPU scan is bit-identical to it); the GPU test shards one index two ways on one device and
merges with pyr_merge_topk_device.
"""
import os
import socket

import numpy as np
import pytest

D, N, NLIST, NPROBE, K, NQ = 32, 3000, 16, 4, 10, 24
BLK = 256  # generator block rows (the sharding unit) for these small sets


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _host_merge(s_parts, l_parts, k):
    """Reference merge for the CPU test: (score desc, label asc), empties (-1) last."""
    Q = s_parts.shape[0]
    out_s = np.full((Q, k), -np.inf, np.float32)
    out_l = np.full((Q, k), -1, np.int64)
    for q in range(Q):
        cand = [(float(s), int(l)) for s, l in zip(s_parts[q].reshape(-1), l_parts[q].reshape(-1)) if l >= 0]
        cand.sort(key=lambda t: (-t[0], t[1]))
        for j, (s, l) in enumerate(cand[:k]):
            out_s[q, j], out_l[q, j] = s, l
    return out_s, out_l


def _shard_search(oracle, data, cents, queries, rank, world):
    """One rank's IVF search over its rows-within-list shard; returns global labels."""
    from pyrope_amd.dist import shard_labels
    labels = shard_labels(len(data), world, rank, BLK)
    rows = data[labels]
    assign = np.array([oracle.find_nearest_centroid(r, cents, oracle.L2) for r in rows], np.int32)
    lrows, order, off = oracle.lists_from_assign(rows, assign, len(cents))
    s, kk, _ = oracle.ivf_search_batch(queries, K, cents, lrows, off, metric=oracle.L2, nprobe=NPROBE)
    lab = np.where(kk >= 0, labels[order[np.maximum(kk, 0)]], -1)
    return s, lab


def _worker(rank, world, port, data, cents, queries, out):
    import torch
    import torch.distributed as dist

    import oracle
    from pyrope_amd.dist import sharded_search

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        def local(q, k):
            s, lab = _shard_search(oracle, data, cents, q.numpy(), rank, world)
            return torch.from_numpy(s), torch.from_numpy(lab)

        def merge(sp, lp, k):
            return tuple(torch.from_numpy(a) for a in _host_merge(sp.numpy(), lp.numpy(), k))

        s, lab = sharded_search(local, merge, torch.from_numpy(queries), K, world)
        np.save(os.path.join(out, f"s{rank}.npy"), s.numpy())
        np.save(os.path.join(out, f"l{rank}.npy"), lab.numpy())
    finally:
        dist.destroy_process_group()


def test_shard_labels_partition():
    from pyrope_amd.dist import shard_blocks, shard_labels
    parts = [shard_labels(103, 4, r, 10) for r in range(4)]
    allp = np.sort(np.concatenate(parts))
    np.testing.assert_array_equal(allp, np.arange(103))
    for r, p in enumerate(parts):
        assert np.all((p // 10) % 4 == r) and np.all(np.diff(p) > 0)
    assert shard_blocks(103, 4, 2, 10) == [(20, 30), (60, 70), (100, 103)]
    assert shard_labels(5, 3, 1, 10).size == 0  # more ranks than blocks: an empty shard


def _oracle_shard(oracle, data, cents, rank, world):
    """One rank's IVF lists over its blocks with the shared quantizer: (labels, lrows, order, off)."""
    from pyrope_amd.dist import shard_labels
    labels = shard_labels(len(data), world, rank, BLK)
    rows = data[labels]
    assign = np.array([oracle.find_nearest_centroid(r, cents, oracle.L2) for r in rows], np.int32)
    lrows, order, off = oracle.lists_from_assign(rows, assign, len(cents))
    return labels, lrows, order, off


def _step_worker(rank, world, port, data, cents, queries, out):
    """bench.py's N > 1 step (pyrope_amd.dist.ShardedIvfStep: buffers allocated once, collectives timed,
    partials merged in the all_gather's [world, Q, k] layout) with the oracle as the scan; two steps
    through the same buffers."""
    import torch
    import torch.distributed as dist

    import oracle
    from pyrope_amd.dist import ShardedIvfStep

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        labels, lrows, order, off = _oracle_shard(oracle, data, cents, rank, world)
        seen = {}

        def probe(qs):  # the coarse ranking of this rank's slice (pyr_index_probe_device)
            return torch.from_numpy(np.stack([oracle.ivf_probe(q, cents, NPROBE) for q in qs.numpy()]))

        def search(qs, probes):  # pyr_index_search_probed_device over this shard
            seen["probes"] = probes.numpy()
            S = np.full((len(qs), K), -np.inf, np.float32)
            Lb = np.full((len(qs), K), -1, np.int64)
            for i, q in enumerate(qs.numpy()):
                s, kk = oracle.ivf_search_probed(q, K, lrows, off, probes[i].numpy())
                S[i, :len(s)] = s
                Lb[i, :len(s)] = labels[order[kk]]
            return torch.from_numpy(S), torch.from_numpy(Lb)

        def merge(sp, lp, k):  # pyr_merge_topk_parts_device(part_major=1): [world, Q, k] as gathered
            assert sp.shape[0] == world
            return tuple(torch.from_numpy(a) for a in _host_merge(sp.numpy().transpose(1, 0, 2),
                                                                 lp.numpy().transpose(1, 0, 2), k))

        step = ShardedIvfStep(len(queries) // world, NPROBE, K, rank, world)
        bufs = (step.probes_all.data_ptr(), step.s_all.data_ptr(), step.l_all.data_ptr())
        step.timing = True
        for _ in range(2):  # the same buffers serve every step
            s, lab = step(torch.from_numpy(queries), probe, search, merge)
        assert (step.probes_all.data_ptr(), step.s_all.data_ptr(), step.l_all.data_ptr()) == bufs
        assert set(step.collective_ms) == {"probe_allgather", "partial_allgather"}
        np.save(os.path.join(out, f"s{rank}.npy"), s.numpy())
        np.save(os.path.join(out, f"l{rank}.npy"), lab.numpy())
        np.save(os.path.join(out, f"p{rank}.npy"), seen["probes"])
    finally:
        dist.destroy_process_group()


def test_gloo_world2_bench_step_equals_unsharded(oracle, tmp_path):
    """the exact N > 1 step bench.py times -- split coarse ranking, probe all_gather,
    per-rank probed search, partial all_gather, merge -- on 2 gloo ranks equals one unsharded search."""
    import torch.multiprocessing as mp

    data = oracle.generate_vectors(N, D, 42)
    queries = oracle.generate_vectors(NQ, D, 1337)
    cents = oracle.kmeans_train(data, NLIST, oracle.L2, 5, 42)
    ref_s, ref_l = _shard_search(oracle, data, cents, queries, 0, 1)
    ref_p = np.stack([oracle.ivf_probe(q, cents, NPROBE) for q in queries])
    port = _free_port()
    mp.start_processes(_step_worker, args=(2, port, data, cents, queries, str(tmp_path)), nprocs=2, join=True,
                       start_method="spawn")
    for r in range(2):
        np.testing.assert_array_equal(np.load(tmp_path / f"p{r}.npy"), ref_p)  # every query's lists on every rank
        np.testing.assert_array_equal(np.load(tmp_path / f"l{r}.npy"), ref_l)
        assert np.array_equal(np.load(tmp_path / f"s{r}.npy").view(np.uint32), ref_s.view(np.uint32))


def test_gloo_world2_sharded_equals_unsharded(oracle, tmp_path):
    import torch.multiprocessing as mp

    data = oracle.generate_vectors(N, D, 42)
    queries = oracle.generate_vectors(NQ, D, 1337)
    cents = oracle.kmeans_train(data, NLIST, oracle.L2, 5, 42)
    # unsharded reference: the whole data set in one index with the same quantizer
    ref_s, ref_l = _shard_search(oracle, data, cents, queries, 0, 1)
    port = _free_port()
    mp.start_processes(_worker, args=(2, port, data, cents, queries, str(tmp_path)), nprocs=2, join=True,
                       start_method="spawn")
    for r in range(2):
        s = np.load(tmp_path / f"s{r}.npy")
        lab = np.load(tmp_path / f"l{r}.npy")
        np.testing.assert_array_equal(lab, ref_l)
        assert np.array_equal(s.view(np.uint32), ref_s.view(np.uint32))


@pytest.mark.gpu
def test_gpu_two_shards_merge_equals_unsharded(hiplib):
    import torch

    from pyrope_amd import IvfFlatVectorIndex, SearchOptions, generate_synthetic, kmeans_train
    from pyrope_amd.dist import merge_device, shard_labels

    n, d, nl = 20000, 128, 64
    data = generate_synthetic(n, d, 42)
    q = generate_synthetic(300, d, 1337)
    cents = kmeans_train(data, nl, 0, 10, 42)
    opts = SearchOptions(nprobe=8)
    full = IvfFlatVectorIndex(d, 0, n_list=nl)
    full.set_centroids(cents)
    full.add_labels(np.arange(n, dtype=np.int64), data)
    full.build()
    ref_s, ref_l, _ = full.search_batch(q, K, opts)
    sp, lp = [], []
    for r in range(2):
        idx = IvfFlatVectorIndex(d, 0, n_list=nl)
        idx.set_centroids(cents)
        lab = shard_labels(n, 2, r, 4096)
        idx.add_labels(lab, data[lab])
        idx.build()
        s, l, _ = idx.search_batch(q, K, opts)
        sp.append(s)
        lp.append(l)
    s_parts = torch.from_numpy(np.stack(sp, 1)).cuda()
    l_parts = torch.from_numpy(np.stack(lp, 1)).cuda()
    s_out, l_out = merge_device(s_parts, l_parts, K)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(l_out.cpu().numpy(), ref_l)
    assert np.array_equal(s_out.cpu().numpy().view(np.uint32), ref_s.view(np.uint32))


@pytest.mark.gpu
def test_gpu_split_coarse_ranking_equals_search(hiplib):
    """bench.py's N > 1 step: each rank ranks the quantizer for its slice of the batch and the
    gathered probe lists feed pyr_index_search_probed_device; same results as the plain search."""
    import torch

    from pyrope_amd import IvfFlatVectorIndex, SearchOptions, generate_synthetic

    n, d, nl, npb = 20000, 128, 64, 8
    data = generate_synthetic(n, d, 42)
    qh = generate_synthetic(300, d, 1337)
    idx = IvfFlatVectorIndex(d, 0, n_list=nl)
    idx.add_labels(np.arange(n, dtype=np.int64), data)
    idx.build()
    opts = SearchOptions(nprobe=npb)
    ref_s, ref_l, _ = idx.search_batch(qh, K, opts)
    q = torch.from_numpy(qh).cuda()
    probes = torch.empty((300, npb), dtype=torch.int32, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    for a, b in [(0, 150), (150, 300)]:  # two "ranks"
        w = idx.probe_device(q[a:b].data_ptr(), b - a, probes[a:b].data_ptr(), stream, opts)
        assert w == npb
    s = torch.empty((300, K), dtype=torch.float32, device="cuda")
    lab = torch.empty((300, K), dtype=torch.int64, device="cuda")
    idx.search_device(q.data_ptr(), 300, K, s.data_ptr(), lab.data_ptr(), 0, stream, opts,
                      d_probes=probes.data_ptr(), nprobe=npb)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(lab.cpu().numpy(), ref_l)
    assert np.array_equal(s.cpu().numpy().view(np.uint32), ref_s.view(np.uint32))


@pytest.mark.gpu
def test_gpu_part_major_merge_equals_query_major(hiplib):
    """pyr_merge_topk_parts_device reads the all_gather layout [world, Q, k] directly: same result as the
    query-major [Q, world, k] merge of the transposed buffer, ties by label."""
    import torch

    from pyrope_amd.dist import merge_device

    rng = np.random.default_rng(5)
    W, Q, k = 8, 777, 10
    s = rng.integers(0, 50, (W, Q, k)).astype(np.float32)  # ties within and across ranks
    lab = rng.permutation(W * Q * k).reshape(W, Q, k).astype(np.int64)
    # every partial list in merge order, (score desc, label asc), as a rank's search returns it
    order = np.lexsort((lab, -s), axis=2)
    s, lab = np.take_along_axis(s, order, 2).copy(), np.take_along_axis(lab, order, 2).copy()
    lab[:, :5, 7:] = -1  # short partial lists
    s[:, :5, 7:] = -np.inf
    sp, lp = torch.from_numpy(s).cuda(), torch.from_numpy(lab).cuda()
    a_s, a_l = merge_device(sp, lp, k, part_major=True)
    b_s, b_l = merge_device(sp.transpose(0, 1).contiguous(), lp.transpose(0, 1).contiguous(), k)
    torch.cuda.synchronize()
    ref_s, ref_l = _host_merge(s.transpose(1, 0, 2), lab.transpose(1, 0, 2), k)
    np.testing.assert_array_equal(a_l.cpu().numpy(), ref_l)
    np.testing.assert_array_equal(b_l.cpu().numpy(), ref_l)
    assert np.array_equal(a_s.cpu().numpy().view(np.uint32), ref_s.view(np.uint32))


def test_rank_memory_plan_at_m8_rank_shape(hiplib):
    """a rank of the 8-GPU M8 run (80M rows / 8 = 10M rows, nlist 8192, the 80,000-query
    weak-scaling batch every rank searches, nprobe 32, k 10) fits one MI355X (288 GB) with room to
    spare, before any rank allocates.  Host arithmetic (pyr_ivf_memory_plan): no GPU needed."""
    from pyrope_amd.dist import rank_memory_plan

    hbm = 288e9
    # list lengths of a 10M-row shard over 8192 lists: mean 1,221; 20,000 covers heavy k-means skew
    ib, wb = rank_memory_plan(128, 10_000_000, 8192, 20_000, 80_000, 32, 10)
    assert 10e9 < ib < 16e9, ib          # ~1.3 kB per row at d = 128 (fp32 blocked + row-major + fp16 tiles)
    assert wb <= 20e9, wb                # candidate regions sliced at 16 GiB + the rest
    assert ib + wb < 0.25 * hbm
    # the I1 single-GPU workload and M8 on one GPU (80M rows, 10,000 queries)
    ib1, wb1 = rank_memory_plan(128, 10_000_000, 1024, 30_000, 10_000, 32, 10)
    assert ib1 + wb1 < 0.1 * hbm
    ib8, wb8 = rank_memory_plan(128, 80_000_000, 8192, 40_000, 10_000, 32, 10)
    assert ib8 + wb8 < 0.5 * hbm
    # the workspace grows with the batch until the 16 GiB region slice caps it
    w_small = rank_memory_plan(128, 10_000_000, 8192, 20_000, 1_000, 32, 10)[1]
    w_big = rank_memory_plan(128, 10_000_000, 8192, 20_000, 1_000_000, 32, 10)[1]
    assert w_small < wb < w_big < 40e9


def test_rank_memory_plan_list_sharded_m8(hiplib):
    """the list-sharded step's rank at the M8 shape (80M rows over 8 ranks, nlist 8192, 10,000
    home queries, every rank searching the 80,000-query batch against its own lists) fits one MI355X with
    room to spare: its whole lists, the replicated 512-row sample of every list, and one step's buffers."""
    from pyrope_amd.dist import rank_memory_plan, rank_memory_plan_lists
    hbm = 288e9
    ib, wb = rank_memory_plan_lists(128, 10_000_000, 8192, 40_000, 10_000, 8, 32, 10)
    ib0, _ = rank_memory_plan(128, 10_000_000, 8192, 40_000, 80_000, 32, 10)
    assert ib0 < ib < ib0 + 8192 * 512 * 1.5e3   # + the sample store (<= 1.5 kB per sampled row)
    assert ib + wb < 0.25 * hbm, (ib, wb)
    # and the build peak of that shard (old + new list store, row temporaries) fits as well
    from pyrope_amd.dist import rank_build_peak_bytes
    bp = rank_build_peak_bytes(128, 10_000_000, 8192, 40_000)
    assert 2 * ib0 < bp < 0.25 * hbm
    # the step's buffers grow with the batch; I1 at 8 ranks (nlist 1024) is far smaller
    ib1, wb1 = rank_memory_plan_lists(128, 1_250_000, 1024, 20_000, 10_000, 8, 32, 10)
    assert ib1 + wb1 < ib + wb
