"""How much slack each constant of the stream filter's upper bound has (measurement only).

The bound every emitted row carries is approx + E_row + E_pair (stream_ub_terms, sample16.hip), built from
five constants: c_bf (the fp16 bilinear rounding of the MFMA product), c_err (fp32 accumulation), c_abs (the
fp16 absolute floor), t (the query's fp16 subnormals) and g (the reference's own fp32 sum).  For each
constant this script multiplies it alone by a falling factor (PYR_EB_<BF|ERR|ABS|T|G>) and counts the rows
whose bound drops below the oracle's exact score (the rows of tests/test_gpu_bounds.py: every visible row of
the scanned lists, PYR_STREAM_EMIT_ALL=1).  The smallest factor with no violation is that constant's slack
(0 = the term is never needed on these data; 1 = no slack).  Also all five together (PYR_EB_*).

    python scripts/bound_slack.py [--out profiles/r5_bounds/slack.json]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

FACTORS = [1.0, 0.5, 0.25, 0.125, 1 / 16, 1 / 64, 1 / 256, 0.0]
CONSTS = ["BF", "ERR", "ABS", "T", "G"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    import oracle
    import test_gpu_bounds as tb
    from pyrope_amd import (BruteForceVectorIndex, IvfFlatVectorIndex, IvfPqVectorIndex, SearchOptions, _lib)
    L = _lib.load()

    def flat(kind, d, metric):
        n, nq = 1500, 6
        x, q = tb.data(kind, n, d, 1), tb.data(kind, nq, d, 2)
        idx = BruteForceVectorIndex(d, metric)
        idx.add_labels(np.arange(n, dtype=np.int64), x, track_ids=False)
        live = np.ones(n, np.uint8)
        ex = []
        for i in range(nq):
            s, kk = oracle.bf_search(x, live, metric, q[i], n)
            out = np.empty(n, np.float32)
            out[kk] = s
            ex.append(out)
        tr = (lambda b: 1.0 + 0.5 * b.astype(np.float64) + (2.0 * d + 256.0) * tb.U) if metric == 2 else None
        return idx, q, None, 2048, ex, tr

    def ivf(kind, d, metric):
        n, nq = 3000, 6
        x, q = tb.data(kind, n, d, 3), tb.data(kind, nq, d, 4)
        idx = IvfFlatVectorIndex(d, metric, n_list=8)
        idx.add_labels(np.arange(n, dtype=np.int64), x, track_ids=False)
        idx.build()
        cents = idx.centroids_array()
        one = np.array([0, n], np.int64)
        ex = []
        for i in range(nq):
            s, kk = oracle.ivf_search(q[i], n, cents[:1], x, one, metric=metric, nprobe=1)
            out = np.empty(n, np.float32)
            out[kk] = s
            ex.append(out)
        return idx, q, SearchOptions(nprobe=3), 4096, ex, None

    def pq(kind, d, m):
        n, nq = 3000, 6
        x, q = tb.data(kind, n, d, 5), tb.data(kind, nq, d, 6)
        idx = IvfPqVectorIndex(d, 0, m=m, k=64, n_list=8)
        idx.add_labels(np.arange(n, dtype=np.int64), x)
        idx.build()
        cb, codes, off, labels, live = idx.pq_state()
        cents = idx.centroids_array()
        ex = []
        for i in range(nq):
            s, kk = oracle.ivfpq_search(q[i], n, cents, codes, off, cb, live, metric=0, nprobe=3)
            out = np.full(n, np.inf, np.float32)
            out[labels[kk]] = s
            ex.append(out)
        return idx, q, SearchOptions(nprobe=3), 4096, ex, None

    configs = []
    for kind in tb.KINDS:
        for d in (128, 768):
            for metric in (0, 1, 2):
                configs.append((f"FLAT {kind} d={d} {['L2', 'IP', 'Cosine'][metric]}", flat, (kind, d, metric)))
            for metric in (0, 1):
                configs.append((f"IVF {kind} d={d} {['L2', 'IP'][metric]}", ivf, (kind, d, metric)))
        for d, m in ((128, 4), (768, 96)):
            configs.append((f"IVF_PQ {kind} d={d} m={m}", pq, (kind, d, m)))

    def violations(idx, q, opts, cap, ex, tr, env):
        old = {k: os.environ.get(k) for k in env}
        os.environ.update({k: str(v) for k, v in env.items()})
        try:
            ub, lab, cnt = tb.emitted(L, idx, q, 10, opts, cap)
        finally:
            for k, v in old.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
        bad, tot, worst = 0, 0, np.inf
        for (l, mg, e) in tb.margins(ub, lab, cnt, lambda i: ex[i], tr):
            bad += int((~(mg >= 0)).sum())
            tot += len(l)
            if len(mg):
                worst = min(worst, float(np.min(mg / np.maximum(1.0, np.abs(e)))))
        return bad, tot, worst

    rows = []
    t0 = time.time()
    for name, mk, a in configs:
        idx, q, opts, cap, ex, tr = mk(*a)
        bad, tot, worst = violations(idx, q, opts, cap, ex, tr, {})
        row = {"config": name, "rows": tot, "violations_at_1": bad, "min_relative_margin": worst, "slack": {}}
        for c in CONSTS + ["ALL"]:
            keys = [f"PYR_EB_{x}" for x in (CONSTS if c == "ALL" else [c])]
            ok = 1.0
            for f in FACTORS[1:]:
                b, _, _ = violations(idx, q, opts, cap, ex, tr, {k_: f for k_ in keys})
                if b:
                    break
                ok = f
            row["slack"][c] = ok
        idx.close()
        rows.append(row)
        print(json.dumps(row), flush=True)
    # per constant: the largest surviving factor over all configurations (the constant's real headroom)
    summary = {c: max(r["slack"][c] for r in rows) for c in CONSTS + ["ALL"]}
    out = {"factors": FACTORS, "configs": rows, "max_factor_needed": summary,
           "violations_at_1": sum(r["violations_at_1"] for r in rows), "seconds": round(time.time() - t0, 1)}
    print(json.dumps({"max_factor_needed": summary, "violations_at_1": out["violations_at_1"]}), flush=True)
    if args.out:
        os.makedirs(os.path.dirname(args.out), exist_ok=True)
        json.dump(out, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
