"""The list-sharded N-GPU step simulated on one GPU (measurement + parity at full size).

Builds the I1 (or M8) data set, assigns every row, and builds ALL `--world` shard indexes on the one GPU
(each owns its size-balanced whole lists, dist.list_owners, plus the replicated sample of every list).
Then it runs the step phase by phase for every rank -- the collectives become tensor copies -- and:
  * times rank `--rank`'s device work: prepare (its home slice), search (all world x nq queries against
    its lists), merge (the world records of its home queries + certificate), rerun (the gathered failures);
  * checks every home's answers against the unsharded index on the same data (ids and score bits);
  * prints the per-rank failure counts and the collectives' byte counts (no collective runs on one GPU);
  * --oracle N: the first N queries of every home against the CPU oracle (IvfFlatVectorIndex.Search restated,
    oracle/oracle.c) over the whole data set -- the check for shapes too large for the unsharded index beside
    the shards (M8: --n 80000000 --nlist 8192 --parity 0 --oracle 25).

    python scripts/rank_shape.py --world 8 [--n 10000000 --nlist 1024 --nprobe 32 --nq 10000 --steps 20]
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--n", type=int, default=10_000_000)
    ap.add_argument("--nlist", type=int, default=1024)
    ap.add_argument("--nprobe", type=int, default=32)
    ap.add_argument("--nq", type=int, default=10_000)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--fcap", type=int, default=256)
    ap.add_argument("--train-rows", type=int, default=10_000_000)
    ap.add_argument("--parity", type=int, default=1, help="compare every home's answers with the unsharded index")
    ap.add_argument("--oracle", type=int, default=0, help="queries per home compared with the CPU oracle")
    ap.add_argument("--determinism", type=int, default=0, help="repeat the unsharded search, the probe ranking and "
                    "the sharded step, and compare (diagnostics)")
    args = ap.parse_args()

    import torch
    torch.cuda.init()
    from pyrope_amd import (IvfFlatVectorIndex, SearchOptions, _lib, assign, generate_synthetic,
                            generate_synthetic_blocked, kmeans_train)
    from pyrope_amd.dist import SAMPLE_ROWS, DeviceShardEngine, list_owners
    L = _lib.load()
    W, R, D, k, nq, F = args.world, args.rank, args.dim, args.k, args.nq, args.fcap
    t = time.time()
    data = generate_synthetic_blocked(0, args.n, D, 42, 65536)
    cents = kmeans_train(data[:min(args.n, args.train_rows)], args.nlist, 0, 10, 42)
    a = np.concatenate([assign(cents, data[i:i + 2_000_000], 0) for i in range(0, args.n, 2_000_000)])
    glen = np.bincount(a, minlength=len(cents))
    owner = list_owners(glen, W)
    order = np.argsort(a, kind="stable")
    off = np.concatenate([[0], np.cumsum(glen)])
    counts = np.minimum(glen, SAMPLE_ROWS)
    srows = np.concatenate([data[order[off[l]:off[l] + counts[l]]] for l in range(len(cents))])
    opts = SearchOptions(nprobe=args.nprobe)

    def index_of(labs):
        ix = IvfFlatVectorIndex(D, 0, n_list=len(cents))
        ix.set_centroids(cents)
        ix.reserve(len(labs))
        for i in range(0, len(labs), 2_000_000):
            ix.add_labels(labs[i:i + 2_000_000], data[labs[i:i + 2_000_000]], track_ids=False)
        ix.build()
        return ix
    shards = []
    for r in range(W):
        ix = index_of(np.nonzero(owner[a] == r)[0].astype(np.int64))
        ix.set_list_samples(srows, counts, glen)
        shards.append(ix)
    Q = W * nq
    qh = generate_synthetic(Q, D, 1337)
    ref = None
    det = {}
    if args.parity:
        full = index_of(np.arange(args.n, dtype=np.int64))
        ref = full.search_batch(qh, k, opts)
        if args.determinism:  # the unsharded answers and probe lists, twice (diagnostics)
            ref2 = full.search_batch(qh, k, opts)
            det["unsharded_repeat_equal"] = bool(np.array_equal(ref[1], ref2[1]) and
                                                 np.array_equal(ref[0].view(np.uint32), ref2[0].view(np.uint32)))
            pr = torch.empty((Q, min(args.nprobe, len(cents))), dtype=torch.int32, device="cuda")
            qd = torch.from_numpy(qh).cuda()
            full.probe_device(qd.data_ptr(), Q, pr.data_ptr(), 0, opts)
            torch.cuda.synchronize()
            full_probes = pr.cpu().numpy().copy()
            full.probe_device(qd.data_ptr(), Q, pr.data_ptr(), 0, opts)
            torch.cuda.synchronize()
            det["probe_repeat_equal"] = bool(np.array_equal(full_probes, pr.cpu().numpy()))
        full.close()
    orc = None
    if args.oracle:  # the oracle's list-major rows (stable by label, the index's storage order) and its answers
        import oracle  # checker only
        xs = data[order]
        sel = np.concatenate([np.arange(h * nq, h * nq + min(args.oracle, nq)) for h in range(W)])
        orc = {}
        t0 = time.time()
        for i in sel:
            os_, ok = oracle.ivf_search(qh[i], k, cents, xs, off, metric=0, nprobe=args.nprobe)
            orc[int(i)] = (os_, order[ok])
        del xs
        print(f"[rank_shape] oracle answers for {len(sel)} queries in {time.time() - t0:.1f}s", flush=True)
    del data, srows
    rows = np.bincount(owner, weights=glen, minlength=W)
    print(f"[rank_shape] world {W}: rank rows max/min {rows.max():.0f}/{rows.min():.0f}, built in "
          f"{time.time() - t:.1f}s", flush=True)

    q = torch.from_numpy(qh).cuda()
    P = min(args.nprobe, len(cents))
    rb = 16 * (k + 1)
    eng = [DeviceShardEngine(ix, k, opts) for ix in shards]
    plans = torch.empty((Q, P + 1), dtype=torch.int32, device="cuda")
    recs = [torch.empty((Q, rb), dtype=torch.uint8, device="cuda") for _ in range(W)]
    out_s = torch.empty((Q, k), dtype=torch.float32, device="cuda")
    out_l = torch.empty((Q, k), dtype=torch.int64, device="cuda")
    fails = torch.zeros((W, 1 + F), dtype=torch.int32, device="cuda")
    rrec = [torch.zeros((W * F, rb), dtype=torch.uint8, device="cuda") for _ in range(W)]
    rec_home = [torch.empty((W, nq, rb), dtype=torch.uint8, device="cuda") for _ in range(W)]
    rrec_home = [torch.empty((W, F, rb), dtype=torch.uint8, device="cuda") for _ in range(W)]

    def hs(h):
        return slice(h * nq, (h + 1) * nq)

    def prepare(r):
        assert eng[r].prepare(q[hs(r)], plans[hs(r)]) == P

    def search(r):
        eng[r].search(q, plans, P, recs[r])

    def merge(h):
        for s in range(W):  # the record all_to_all's output at home h
            rec_home[h][s].copy_(recs[s][hs(h)])
        eng[h].merge(rec_home[h], out_s[hs(h)], out_l[hs(h)], fails[h])

    def rerun(r):
        eng[r].rerun(q, plans, P, fails, nq, rrec[r])

    def finish(h):
        for s in range(W):
            rrec_home[h][s].copy_(rrec[s][h * F:(h + 1) * F])
        eng[h].merge_rerun(rrec_home[h], fails[h], out_s[hs(h)], out_l[hs(h)])

    def full_step():
        for r in range(W):
            prepare(r)
        for r in range(W):
            search(r)
        for h in range(W):
            merge(h)
        for r in range(W):
            rerun(r)
        for h in range(W):
            finish(h)

    full_step()
    torch.cuda.synchronize()
    if args.determinism and args.parity:
        P0 = min(args.nprobe, len(cents))
        hp = plans[:, :P0].cpu().numpy()
        det["plan_probes_equal_unsharded"] = bool(np.array_equal(np.sort(hp, 1), np.sort(full_probes, 1)))
        det["plan_probes_differing_queries"] = int((np.sort(hp, 1) != np.sort(full_probes, 1)).any(1).sum())
        s1, l1 = out_s.cpu().numpy().copy(), out_l.cpu().numpy().copy()
        plan1 = plans.cpu().numpy().copy()
        recs1 = [r_.cpu().numpy().copy() for r_ in recs]
        fails1 = fails.cpu().numpy().copy()
        full_step()
        torch.cuda.synchronize()
        det["sharded_repeat_equal"] = bool(np.array_equal(l1, out_l.cpu().numpy()) and
                                           np.array_equal(s1.view(np.uint32), out_s.cpu().numpy().view(np.uint32)))
        hp2 = plans[:, :P0].cpu().numpy()
        det["plan_repeat_equal"] = bool(np.array_equal(hp, hp2))
        plan2 = plans.cpu().numpy()
        det["plan_thr_repeat_equal"] = bool(np.array_equal(plan1.view(np.uint32), plan2.view(np.uint32)))
        det["plan_thr_nan"] = int(np.isnan(plan1[:, P0].view(np.float32)).sum())
        rdiff = [int((recs1[r_] != recs[r_].cpu().numpy()).any(1).sum()) for r_ in range(W)]
        det["record_rows_differing_per_rank"] = rdiff
        det["fails_repeat_equal"] = bool(np.array_equal(fails1, fails.cpu().numpy()))
        bad = np.nonzero((l1 != out_l.cpu().numpy()).any(1))[0]
        if len(bad):
            b = int(bad[0])
            dr = [r_ for r_ in range(W) if (recs1[r_][b] != recs[r_][b].cpu().numpy()).any()]

            def dec(raw):  # k ShardEntry {int64 label, float score, int32 list} + trailer {float bound, int32 n}
                ent = [(int(raw[16 * i:16 * i + 8].view(np.int64)[0]), float(raw[16 * i + 8:16 * i + 12].view(np.float32)[0]),
                        int(raw[16 * i + 12:16 * i + 16].view(np.int32)[0])) for i in range(k)]
                tr = (float(raw[16 * k:16 * k + 4].view(np.float32)[0]), int(raw[16 * k + 4:16 * k + 8].view(np.int32)[0]))
                return {"ent": ent, "trailer": tr}
            det["first_differing"] = {"q": b, "l1": l1[b].tolist(), "l2": out_l.cpu().numpy()[b].tolist(),
                                      "recs_differ_on_ranks": dr,
                                      "rec1": [dec(recs1[r_][b]) for r_ in dr], "rec2": [dec(recs[r_][b].cpu().numpy()) for r_ in dr]}
        out_s.copy_(torch.from_numpy(s1))
        out_l.copy_(torch.from_numpy(l1))
    per = np.bincount(owner[plans[:, :P].cpu().numpy().ravel()], minlength=W)
    res = {"determinism": det, "world": W, "rank": R, "rows": int(rows[R]), "lists": int((owner == R).sum()), "queries_all": Q,
           "queries_home": nq, "nprobe": P, "failures_per_home": fails[:, 0].cpu().tolist(),
           "pairs_per_rank": per.tolist(), "pairs_max_over_mean": round(float(per.max() / per.mean()), 4),
           "rows_per_rank": rows.astype(np.int64).tolist()}
    if ref is not None:
        s_, l_ = out_s.cpu().numpy(), out_l.cpu().numpy()
        res["parity"] = {"queries": Q, "ids_equal": bool(np.array_equal(l_, ref[1])),
                         "scores_bit_identical": bool(np.array_equal(s_.view(np.uint32), ref[0].view(np.uint32)))}
        bad = np.nonzero((l_ != ref[1]).any(1) | (s_.view(np.uint32) != ref[0].view(np.uint32)).any(1))[0]
        if len(bad):  # which queries differ, and whether their home listed them as certificate failures
            fl = fails.cpu().numpy()
            failed = {h * nq + int(i) for h in range(W) for i in fl[h, 1:1 + min(int(fl[h, 0]), F)]}
            res["parity"]["differing"] = [{"q": int(b), "home": int(b // nq), "failed": int(b) in failed,
                                           "got": l_[b].tolist(), "ref": ref[1][b].tolist()} for b in bad[:4]]
            res["parity"]["n_differing"] = int(len(bad))
    if orc is not None:
        s_, l_ = out_s.cpu().numpy(), out_l.cpu().numpy()
        ok = [bool(np.array_equal(l_[i][:len(kk)], kk) and np.array_equal(s_[i][:len(ss)].view(np.uint32), ss.view(np.uint32)))
              for i, (ss, kk) in orc.items()]
        res["oracle_sample"] = {"queries": len(ok), "ids_and_bits_equal": all(ok), "equal": int(sum(ok))}
    # rank R's device phases, each timed over --steps repetitions (the other ranks' records stay as computed)
    phases = {"prepare": lambda: prepare(R), "search": lambda: search(R), "merge": lambda: merge(R)}
    # the step skips the re-run (its phases and its all_to_all) when no home has a failure (dist.ListShardedIvf)
    if int(fails[:, 0].max()) > 0:
        phases["rerun"] = lambda: (rerun(R), finish(R))
    ev = {}
    for name, f in phases.items():
        f()
        a0, b0 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a0.record()
        for _ in range(args.steps):
            f()
        b0.record()
        b0.synchronize()
        ev[name] = a0.elapsed_time(b0) / args.steps
    res["phase_ms"] = {k_: round(v, 4) for k_, v in ev.items()}
    res["rank_step_ms_no_collectives"] = round(sum(ev.values()), 4)
    L.pyr_profile_reset()
    L.pyr_profile_enable(1)
    for f in phases.values():
        f()
    torch.cuda.synchronize()
    L.pyr_profile_enable(0)
    names = {0: "coarse", 1: "work_lists", 9: "sample", 2: "list_scan", 4: "merge", 7: "refine", 8: "exact_rerun"}
    prof = {}
    for ph, name in names.items():
        ms, calls, work = C.c_double(), C.c_int64(), C.c_int64()
        L.pyr_profile_get(ph, C.byref(ms), C.byref(calls), C.byref(work))
        if calls.value:
            prof[name] = round(ms.value, 4)
    res["library_phases_ms"] = prof
    res["collective_bytes_per_rank"] = {"plan_allgather_recv": Q * (P + 1) * 4, "record_alltoall_send": Q * rb,
                                        "fail_allgather_recv": W * (1 + F) * 4, "rerun_alltoall_send": W * F * rb}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
