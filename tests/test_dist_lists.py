"""List-sharded multi-GPU IVF_FLAT (pyrope_amd/dist.py ListShardedIvf) on CPU ranks.

The orchestration -- the row exchange that gives every rank WHOLE lists in label order, the replicated
list samples, and the step (plan all_gather, record all_to_all, merge + certificate, fail-list all_gather,
exact re-run, re-run all_to_all) -- runs on world-2/3 gloo groups with an oracle-backed engine that keeps
the device engine's record semantics (exact local top-k + the bound of the rows left out):
the step's answers must equal the unsharded index's (oracle/oracle.c IVF search over the same probes),
ties included, whatever the thresholds do -- some queries are given thresholds that force the
certificate to fail, so the re-run path answers them.

The reference loop being split across ranks: IvfFlatVectorIndex.cs:198-218.
"""
import os
import socket

import numpy as np
import pytest

D, N, NLIST, NPROBE, K, NQ = 16, 2400, 12, 4, 10, 12   # NQ queries per rank
BLK = 200                                             # generator block rows (the sharding unit)
K1 = 16


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


ENTRY = np.dtype([("label", "<i8"), ("score", "<f4"), ("list", "<i4")])
TRAIL = np.dtype([("bound", "<f4"), ("n", "<i4"), ("pad", "<i8")])


def _rec_view(t, k=K):
    """uint8 torch tensor [..., 16 (k + 1)] -> (entries [..., k], trailer [...]) numpy views."""
    a = t.numpy()
    shape = a.shape[:-1]
    flat = a.reshape(-1, 16 * (k + 1))
    ent = flat[:, :16 * k].copy().view(ENTRY).reshape(shape + (k,))
    tr = flat[:, 16 * k:].copy().view(TRAIL).reshape(shape)
    return ent, tr


def _rec_write(t, i, ent, tr):
    flat = t.numpy().reshape(-1, t.shape[-1])
    flat[i, :ent.nbytes] = np.frombuffer(ent.tobytes(), np.uint8)
    flat[i, ent.nbytes:] = np.frombuffer(tr.tobytes(), np.uint8)


def _better_key(s, lst, lab):
    return (-s, lst, lab)


class CpuEngine:
    """The per-rank operations of the step on the oracle (exact scores stand in for the fp16 bounds)."""

    def __init__(self, oracle, cents, lists, k, thr_of):
        self.O, self.cents, self.lists, self.k, self.thr_of = oracle, cents, lists, k, thr_of
        self.reruns = 0

    def _scores(self, q, probes):
        """(score, list, label) of every row of the owned lists among probes."""
        out = []
        for l in probes:
            rows, labs = self.lists.get(int(l), (None, None))
            if rows is None or len(rows) == 0:
                continue
            s, kk = self.O.ivf_search_probed(q, len(rows), rows, np.array([0, len(rows)]), np.array([0], np.int32))
            out += [(float(sc), int(l), int(labs[j])) for sc, j in zip(s, kk)]
        return out

    def prepare(self, q_home, plan):
        for i, q in enumerate(q_home.numpy()):
            pr = self.O.ivf_probe(q, self.cents, NPROBE)
            plan.numpy()[i, :NPROBE] = pr
            plan.numpy()[i, NPROBE] = np.float32(self.thr_of(q)).view(np.int32)
        return NPROBE

    def _record(self, cands, bound):
        cands.sort(key=lambda t: _better_key(*t))
        ent = np.zeros(self.k, ENTRY)
        ent["label"], ent["score"], ent["list"] = -1, -np.inf, 0x7FFFFFFF
        for j, (s, lst, lab) in enumerate(cands[:self.k]):
            ent[j] = (lab, s, lst)
        tr = np.zeros(1, TRAIL)
        tr["bound"], tr["n"] = bound, min(len(cands), self.k)
        return ent, tr

    def search(self, q_all, plan_all, width, rec):
        for i, q in enumerate(q_all.numpy()):
            pr = plan_all.numpy()[i, :width]
            T = plan_all.numpy()[i, width:width + 1].view(np.float32)[0]
            allr = self._scores(q, pr)
            cands = [t for t in allr if t[0] >= T]           # "emitted": bound >= T
            bound = -np.inf if len(cands) == len(allr) else float(T)
            if len(cands) > K1:                              # the refine's depth: the K1-th bound covers the rest
                cands.sort(key=lambda t: _better_key(*t))
                bound = max(bound, cands[K1 - 1][0])
                cands = cands[:K1]
            _rec_write(rec, i, *self._record(cands, bound))

    def merge(self, rec_parts, out_s, out_l, fail, qsel=None):
        ent, tr = _rec_view(rec_parts)
        world, n = ent.shape[0], ent.shape[1]
        fcap = fail.shape[0] - 1 if fail is not None else 0
        nfail = 0
        for i in range(n if qsel is None else min(int(qsel[0]), n)):  # (the device merge's cap = its records)
            q = i if qsel is None else int(qsel[1 + i])
            allc = [(float(e["score"]), int(e["list"]), int(e["label"])) for s in range(world)
                    for e in ent[s, i][:int(tr[s, i]["n"])]]
            allc.sort(key=lambda t: _better_key(*t))
            top = allc[:self.k]
            out_s.numpy()[q] = -np.inf
            out_l.numpy()[q] = -1
            for j, (s, _, lab) in enumerate(top):
                out_s.numpy()[q, j], out_l.numpy()[q, j] = s, lab
            b = max(float(tr[s, i]["bound"]) for s in range(world))
            ok = b == -np.inf or (len(top) == self.k and top[-1][0] > b)
            if fail is not None and not ok:
                if nfail < fcap:
                    fail.numpy()[1 + nfail] = q
                nfail += 1
        if fail is not None:
            fail.numpy()[0] = nfail

    def rerun(self, q_all, plan_all, width, fails_all, nq_home, rec):
        fa = fails_all.numpy()
        world, f1 = fa.shape
        for s in range(world):
            for j in range(min(int(fa[s, 0]), f1 - 1)):
                q = s * nq_home + int(fa[s, 1 + j])
                self.reruns += 1
                _rec_write(rec, s * (f1 - 1) + j,
                           *self._record(self._scores(q_all.numpy()[q], plan_all.numpy()[q, :width]), -np.inf))

    def merge_rerun(self, rec_parts, fail_home, out_s, out_l):
        self.merge(rec_parts, out_s, out_l, None, qsel=fail_home.numpy())


def _chunks(data, rank, world, per_round=2):
    """Rank r's generator blocks b % world == r in rounds of per_round blocks (round i of every rank covers
    one contiguous range of blocks: the receivers' label order is the unsharded list order)."""
    from pyrope_amd.dist import shard_blocks
    blocks = shard_blocks(len(data), world, rank, BLK)

    def gen():
        for i in range(0, len(blocks), per_round):
            labs = np.concatenate([np.arange(a, b, dtype=np.int64) for a, b in blocks[i:i + per_round]])
            yield labs, data[labs]
    return gen


def _worker(rank, world, port, data, cents, queries, thr, out, fcap):
    import torch

    import oracle
    from pyrope_amd.dist import Comm, ListShardedIvf, exchange_rows, gather_samples

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        comm = Comm(world)
        got = {}

        def add(labs, rows):
            for lab, row in zip(labs, rows):
                got.setdefault(int(lab), row)
            add.order.extend(labs.tolist())
        add.order = []

        def assign_fn(c, x):
            return np.array([oracle.find_nearest_centroid(r, c, oracle.L2) for r in x], np.int32)

        glen, owner, samples = exchange_rows(comm, rank, world, _chunks(data, rank, world), cents, 0,
                                             add=add, assign_fn=assign_fn)
        srows, scounts = gather_samples(comm, rank, world, glen, owner, samples, D)
        # this rank's lists, rows in arrival (label) order
        asg = np.array([oracle.find_nearest_centroid(data[lab], cents, oracle.L2) for lab in add.order], np.int32)
        lists = {}
        for l in np.unique(asg):
            labs = np.array([lab for lab, a in zip(add.order, asg) if a == l], np.int64)
            lists[int(l)] = (data[labs], labs)
        thr_map = {tuple(q.tolist()): t for q, t in zip(queries, thr)}
        eng = CpuEngine(oracle, cents, lists, K, lambda q: thr_map[tuple(q.tolist())])
        step = ListShardedIvf(eng, comm, NQ, K, NPROBE, rank, world, fcap=fcap)
        step.timing = True
        for _ in range(2):
            s, lab = step(torch.from_numpy(queries))
        np.save(os.path.join(out, f"s{rank}.npy"), s.numpy())
        np.save(os.path.join(out, f"l{rank}.npy"), lab.numpy())
        np.save(os.path.join(out, f"order{rank}.npy"), np.array(add.order, np.int64))
        np.save(os.path.join(out, f"own{rank}.npy"), owner)
        np.save(os.path.join(out, f"glen{rank}.npy"), glen)
        np.save(os.path.join(out, f"srows{rank}.npy"), srows)
        np.save(os.path.join(out, f"scounts{rank}.npy"), scounts)
        np.save(os.path.join(out, f"meta{rank}.npy"), np.array([eng.reruns, step.stats["extra_rounds"],
                                                                step.max_fail]))
        names = {"plan_allgather", "record_alltoall", "fail_allgather", "rerun_alltoall"}
        if step.stats["extra_rounds"]:
            names.add("fail_full_allgather")
        assert set(step.collective_ms) == names
    finally:
        dist.destroy_process_group()


def _setup(oracle):
    data = oracle.generate_vectors(N, D, 42)
    cents = oracle.kmeans_train(data, NLIST, oracle.L2, 5, 42)
    return data, cents


def _unsharded(oracle, data, cents, queries):
    assign = np.array([oracle.find_nearest_centroid(r, cents, oracle.L2) for r in data], np.int32)
    lrows, order, off = oracle.lists_from_assign(data, assign, len(cents))
    S = np.full((len(queries), K), -np.inf, np.float32)
    L = np.full((len(queries), K), -1, np.int64)
    for i, q in enumerate(queries):
        s, kk = oracle.ivf_search(q, K, cents, lrows, off, metric=oracle.L2, nprobe=NPROBE)
        S[i, :len(s)], L[i, :len(s)] = s, order[kk]
    return S, L, assign, order, off


@pytest.mark.parametrize("world,fcap", [(2, 8), (3, 8), (2, 1), (3, 2)])
def test_list_sharded_step_equals_unsharded(oracle, tmp_path, world, fcap):
    """fcap 8 holds every home's failures in the fixed re-run round; fcap 1 / 2 is smaller than a home's
    failure count (NQ / 3 = 4), so the step runs further rounds -- every failure must still come back exact."""
    import torch.multiprocessing as mp

    from pyrope_amd.dist import SAMPLE_ROWS, list_owners
    data, cents = _setup(oracle)
    queries = oracle.generate_vectors(NQ * world, D, 1337)
    ref_s, ref_l, assign, order, off = _unsharded(oracle, data, cents, queries)
    # thresholds: 30th best (certificate holds), 4th best (fails: re-run), -inf (all candidates)
    lrows = data[order]
    thr = np.empty(len(queries), np.float32)
    for i, q in enumerate(queries):
        s40, _ = oracle.ivf_search(q, 40, cents, lrows, off, metric=oracle.L2, nprobe=NPROBE)
        thr[i] = [s40[29], s40[3], -np.inf][i % 3]
    port = _free_port()
    mp.start_processes(_worker, args=(world, port, data, cents, queries, thr, str(tmp_path), fcap), nprocs=world,
                       join=True, start_method="spawn")
    glen = np.bincount(assign, minlength=len(cents))
    owner = list_owners(glen, world)
    reruns = 0
    for r in range(world):
        np.testing.assert_array_equal(np.load(tmp_path / f"glen{r}.npy"), glen)
        np.testing.assert_array_equal(np.load(tmp_path / f"own{r}.npy"), owner)
        # whole lists, rows in label order
        got = np.load(tmp_path / f"order{r}.npy")
        want = np.sort(np.nonzero(owner[assign] == r)[0])
        np.testing.assert_array_equal(got, want)
        # every rank holds the first SAMPLE_ROWS rows of every list in list order
        cnt = np.minimum(glen, SAMPLE_ROWS)
        np.testing.assert_array_equal(np.load(tmp_path / f"scounts{r}.npy"), cnt)
        exp = np.concatenate([data[order[off[l]:off[l] + cnt[l]]] for l in range(len(cents))])
        np.testing.assert_array_equal(np.load(tmp_path / f"srows{r}.npy"), exp)
        # the step's answers for this rank's home queries
        s, lab = np.load(tmp_path / f"s{r}.npy"), np.load(tmp_path / f"l{r}.npy")
        np.testing.assert_array_equal(lab, ref_l[r * NQ:(r + 1) * NQ])
        assert np.array_equal(s.view(np.uint32), ref_s[r * NQ:(r + 1) * NQ].view(np.uint32))
        meta = np.load(tmp_path / f"meta{r}.npy")
        reruns += int(meta[0])
        nf = NQ // 3  # the forced failures per home
        assert meta[2] == nf
        assert meta[1] == (nf - 1) // fcap  # rounds past the fixed one
    # every forced failure (a third of the queries) was re-run exactly, on every rank, in both steps
    assert reruns == 2 * world * (NQ * world // 3)


def test_list_owners_balance():
    from pyrope_amd.dist import list_owners
    rng = np.random.default_rng(3)
    lens = rng.integers(1, 5000, 1024)
    for w in (1, 2, 3, 8):
        o = list_owners(lens, w)
        assert o.min() >= 0 and o.max() < w
        loads = np.bincount(o, weights=lens, minlength=w)
        assert loads.max() - loads.min() <= lens.max()  # LPT: within one list of balanced
        np.testing.assert_array_equal(o, list_owners(lens, w))  # deterministic
