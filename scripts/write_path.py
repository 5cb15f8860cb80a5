"""The row-at-a-time write path (BruteForceVectorIndex.cs:133-222, DeltaVectorIndex.cs:29-56).

VEC.ADD writes one vector per call into the Delta head (a FLAT index).  This script measures that
granularity on the device:

  1. a FLAT L2 head bulk-loaded with --base rows (d=128), then --adds single-row adds through the C ABI
     (pyr_index_add, one row per call: the small-batch path of RowStore::write -- one pinned staging copy,
     one fused kernel, no host synchronization), with a --qb-query search every --every adds; adds/s over
     the time spent in the add calls, and over the whole loop;
  2. the interleaved searches and a final batch compared with the CPU oracle (BruteForceVectorIndex.Search
     restated, oracle/oracle.c) over the rows written so far: ids and score bits;
  3. a head whose FIRST write was one row (its fp16 tiles centred on that row until re-centred): the
     emitted rows per query and the certificate re-runs of a 1,000-query batch, with the center following
     the rows (default: re-centred each time the store doubles, and at build) vs frozen at the first row
     (PYR_FROZEN_CENTER=1, round 4's behaviour) vs a bulk-loaded head.

    python scripts/write_path.py [--base 1000000 --adds 100000 --every 5000]
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--base", type=int, default=1_000_000)
    ap.add_argument("--adds", type=int, default=100_000)
    ap.add_argument("--every", type=int, default=5_000)
    ap.add_argument("--qb", type=int, default=4)
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--check", type=int, default=1, help="compare searches with the CPU oracle")
    ap.add_argument("--one-row-head", type=int, default=200_000, help="rows of the head whose first write is one row")
    args = ap.parse_args()
    import oracle  # checker only
    from pyrope_amd import BruteForceVectorIndex, _lib, generate_synthetic
    L = _lib.load()
    D, k = args.dim, 10
    out = {"dim": D, "base_rows": args.base, "adds": args.adds}
    total = args.base + args.adds
    x = generate_synthetic(total, D, 42)
    lab = np.arange(total, dtype=np.int64)
    head = BruteForceVectorIndex(D, 0)
    head.reserve(total)
    t = time.time()
    for a in range(0, args.base, 65536):
        e = min(args.base, a + 65536)
        head.add_labels(lab[a:e], x[a:e], track_ids=False)
    print(f"[write] bulk-loaded {args.base} rows in {time.time() - t:.1f}s", flush=True)
    qs = generate_synthetic(4096, D, 1337)
    h = head._h
    pf, pl = x.ctypes.data, lab.ctypes.data
    FP, LP = C.POINTER(C.c_float), C.POINTER(C.c_int64)
    checks, add_s = [], 0.0
    t_loop = time.perf_counter()
    qi = 0
    for a in range(args.base, total, args.every):
        e = min(total, a + args.every)
        t0 = time.perf_counter()
        for i in range(a, e):  # one row per call, as VEC.ADD issues them
            rc = L.pyr_index_add(h, C.cast(pf + i * D * 4, FP), 1, C.cast(pl + i * 8, LP))
            if rc:
                raise RuntimeError(L.pyr_last_error())
        add_s += time.perf_counter() - t0
        q = qs[qi:qi + args.qb]
        qi += args.qb
        s, l, _ = head.search_batch(q, k)
        if args.check:
            live = np.ones(e, np.uint8)
            for j in range(len(q)):
                os_, ok = oracle.bf_search(x[:e], live, 0, q[j], k)
                checks.append(bool(np.array_equal(ok, l[j]) and np.array_equal(os_.view(np.uint32), s[j].view(np.uint32))))
    loop_s = time.perf_counter() - t_loop
    out["adds_per_s_in_add_calls"] = args.adds / add_s
    out["adds_per_s_with_searches"] = args.adds / loop_s
    out["interleaved_searches"] = {"queries": len(checks), "bit_identical_to_oracle": all(checks) if checks else None}
    print(f"[write] {args.adds} single-row adds: {out['adds_per_s_in_add_calls']:,.0f}/s in the add calls, "
          f"{out['adds_per_s_with_searches']:,.0f}/s with {len(checks)} interleaved query searches "
          f"(oracle-identical: {out['interleaved_searches']['bit_identical_to_oracle']})", flush=True)
    # the Python API at the same granularity (numpy conversion + id map per call)
    py = BruteForceVectorIndex(D, 0)
    n_py = min(20_000, args.adds)
    t0 = time.perf_counter()
    for i in range(n_py):
        py.add_labels(lab[i:i + 1], x[i:i + 1], track_ids=False)
    out["python_add_labels_per_s"] = n_py / (time.perf_counter() - t0)
    py.close()
    head.close()

    # 3. a head whose first write was one row
    def one_row_head(env, n, bulk=False):
        old = {kk: os.environ.get(kk) for kk in env}
        os.environ.update(env)
        try:
            ix = BruteForceVectorIndex(D, 0)
            ix.reserve(n)
            if bulk:
                for a in range(0, n, 65536):
                    ix.add_labels(lab[a:min(n, a + 65536)], x[a:min(n, a + 65536)], track_ids=False)
            else:
                ix.add_labels(lab[:1], x[:1], track_ids=False)  # the first write: one row
                for a in range(1, n, 64):  # then small writes (64 rows per call)
                    ix.add_labels(lab[a:min(n, a + 64)], x[a:min(n, a + 64)], track_ids=False)
            q = qs[:1000]
            L.pyr_profile_reset()
            L.pyr_profile_enable(1)
            s, l, _ = ix.search_batch(q, k)
            L.pyr_profile_enable(0)
            ms, calls, work = C.c_double(), C.c_int64(), C.c_int64()
            L.pyr_profile_get(8, C.byref(ms), C.byref(calls), C.byref(work))
            cap = int(os.environ.get("PYR_STREAM_CAP", "2048"))
            ub = np.empty((len(q), cap), np.float32)
            lb = np.empty((len(q), cap), np.int64)
            cnt = np.empty(len(q), np.int32)
            rc = L.pyr_index_debug_candidates(ix._h, len(q), cap, ub.ctypes.data_as(C.c_void_p),
                                              lb.ctypes.data_as(C.c_void_p), cnt.ctypes.data_as(C.c_void_p))
            emitted = float(cnt.mean()) if rc == 0 else None
            same = None
            if args.check:
                live = np.ones(n, np.uint8)
                same = all(np.array_equal(oracle.bf_search(x[:n], live, 0, q[j], k)[1], l[j]) for j in range(0, 1000, 97))
            ix.close()
            return {"emitted_rows_per_query": emitted, "reruns": work.value, "queries": len(q),
                    "ids_equal_oracle_sample": same}
        finally:
            for kk, v in old.items():
                if v is None:
                    os.environ.pop(kk, None)
                else:
                    os.environ[kk] = v
    n1 = args.one_row_head
    out["one_row_first_write"] = {
        "rows": n1,
        "recentred": one_row_head({}, n1),
        "frozen_center": one_row_head({"PYR_FROZEN_CENTER": "1"}, n1),
        "bulk_loaded": one_row_head({}, n1, bulk=True),
    }
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
