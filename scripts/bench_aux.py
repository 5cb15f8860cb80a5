#!/usr/bin/env python3
"""Secondary measurements for DESIGN.md (not the driver's bench line; bench.py is that).

    python scripts/bench_aux.py flat  [--n 1000000 --nq 10000 --metric 0|1]
    python scripts/bench_aux.py ivfpq [--n 3200000 --dim 768 --nlist 256 --m 96 --nprobe 64 --nq 10000]

flat   BASELINE.json configs[1]: FLAT d=128 N=1M Q=10k (L2 and IP), HBM-resident batch.
ivfpq  IVF_PQ d=768 m=96 k=256 nprobe=64 with lists of ~12.5k rows -- the per-query work of
       configs[3] (N=50M, nlist=4096: 64 x 12.2k rows x 96 lookups per query) on a
       smaller index (N/nlist kept, nlist smaller) so that the box builds it in minutes.

Prints one JSON line per run: QPS, per-phase HIP-event times, the dominant kernel's
algorithmic rate, and parity of a query sample against the CPU oracle (test infrastructure,
outside the timed region).
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PH = {0: "coarse", 1: "work_lists", 2: "list_scan", 3: "buffer_scan", 4: "merge", 5: "flat_scan", 6: "pq_scan",
      7: "refine", 8: "exact_rerun"}


def log(*a):
    print("[aux]", *a, file=sys.stderr, flush=True)


def timed(idx, q, Q, k, opts, steps, warmup, L):
    import torch
    dev = q.device
    s = torch.empty((Q, k), dtype=torch.float32, device=dev)
    lab = torch.empty((Q, k), dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream().cuda_stream

    def step():
        idx.search_device(q.data_ptr(), Q, k, s.data_ptr(), lab.data_ptr(), 0, stream, opts)

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    L.pyr_profile_reset()
    L.pyr_profile_enable(1)
    step()
    torch.cuda.synchronize()
    L.pyr_profile_enable(0)
    phases = {}
    for ph, name in PH.items():
        ms, calls, work = C.c_double(), C.c_int64(), C.c_int64()
        L.pyr_profile_get(ph, C.byref(ms), C.byref(calls), C.byref(work))
        if calls.value:
            phases[name] = {"ms": round(ms.value, 4), "work": work.value}
    return Q * steps / el, el / steps * 1e3, phases, s.cpu().numpy(), lab.cpu().numpy()


def pq_roofline(lookups_per_s):
    """LDS-gather roofline of pq_adc4: one ds_read_b128 serves 64 rows x 4 queries = 256
    (query, row, subspace) lookups in 4 LDS cycles (16-lane groups, MI355X_MICROARCH.md LDS table) when
    conflict-free: 64 lookups/clk/CU x 256 CUs x 2.4 GHz.  Random 8-bit codes put a group's 16 lanes on
    16 bank slots (code mod 16) at random: the expected busiest slot holds 3.08 of them (simulated), so
    a random gather costs ~3.08x the conflict-free cycles -- `random_bank_peak`."""
    peak = 64 * 256 * 2.4e9 / 1e12
    rand = peak / 3.08
    ach = lookups_per_s / 1e12
    return {"bound": "lds", "achieved": ach, "peak": peak, "unit": "T lookups/s", "frac": ach / peak,
            "random_bank_peak": rand, "frac_of_random_bank_peak": ach / rand,
            "note": "peak = conflict-free ds_read_b128 gathers (64 lookups/clk/CU); random_bank_peak divides it "
                    "by the expected 3.08-way bank-slot collision of 16 random codes"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("workload", choices=["flat", "ivfpq"])
    ap.add_argument("--n", type=int, default=0)
    ap.add_argument("--dim", type=int, default=0)
    ap.add_argument("--nq", type=int, default=10000)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--metric", type=int, default=0)
    ap.add_argument("--quant", action="store_true", help="flat: EnableQuantization (8-bit search mode)")
    ap.add_argument("--nlist", type=int, default=256)
    ap.add_argument("--m", type=int, default=96)
    ap.add_argument("--nprobe", type=int, default=64)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--check", type=int, default=20, help="queries compared with the CPU oracle")
    ap.add_argument("--recall-queries", type=int, default=0, help="ivfpq: recall@k vs exact FLAT over all N rows")
    ap.add_argument("--train-rows", type=int, default=0,
                    help="ivfpq: train the quantizers on the first N rows and stream the rest (0 = all rows)")
    ap.add_argument("--cpu-seconds", type=float, default=0.0,
                    help="flat: also time the CPU restatement (oracle, one query per thread, every usable CPU)")
    ap.add_argument("--sweep", default="", help="env settings run one after another on the same index, "
                                                 "e.g. 'PYR_PQ_THREADS=1024|PYR_PQ_ABLATE=1' (timing only)")
    a = ap.parse_args()

    def heartbeat():  # long host-side steps of a 50M-row build print nothing for minutes (the harness's hang guard)
        t0 = time.time()
        while True:
            time.sleep(60)
            print(f"[aux] {time.time() - t0:.0f} s", file=sys.stderr, flush=True)

    import threading
    threading.Thread(target=heartbeat, daemon=True).start()

    import torch
    from pyrope_amd import (BruteForceVectorIndex, IvfPqVectorIndex, SearchOptions, _lib, generate_synthetic)
    from pyrope_amd.build import build
    build()
    L = _lib.load()
    torch.cuda.set_device(0)
    import oracle  # parity check of a sample only

    def run_sweep(idx, q, opts, s, lab):
        """time the same index under each env setting of --sweep (results compared with the default's)"""
        for setting in [x for x in a.sweep.split("|") if x]:
            kv = dict(t.split("=") for t in setting.split(","))
            old = {k_: os.environ.get(k_) for k_ in kv}
            os.environ.update(kv)
            qps2, ms2, ph2, s2, l2 = timed(idx, q, a.nq, a.k, opts, a.steps, a.warmup, L)
            for k_, v in old.items():
                if v is None:
                    os.environ.pop(k_, None)
                else:
                    os.environ[k_] = v
            print(json.dumps({"sweep": setting, "qps": qps2, "ms_per_step": ms2,
                              "phases_ms": {k_: v["ms"] for k_, v in ph2.items()},
                              "same_results": bool(np.array_equal(l2, lab) and np.array_equal(s2.view(np.uint32),
                                                                                             s.view(np.uint32)))}),
                  flush=True)

    if a.workload == "flat":
        n, d = a.n or 1_000_000, a.dim or 128
        x = generate_synthetic(n, d, 42)
        qh = generate_synthetic(a.nq, d, 1337)
        idx = BruteForceVectorIndex(d, a.metric)
        if a.quant:
            idx.enable_quantization = True
        idx.add_labels(np.arange(n, dtype=np.int64), x)
        q = torch.from_numpy(qh).cuda()
        qps, ms, phases, s, lab = timed(idx, q, a.nq, a.k, None, a.steps, a.warmup, L)
        run_sweep(idx, q, None, s, lab)
        ok = True
        for i in np.linspace(0, a.nq - 1, a.check).astype(int):
            if a.quant:
                os_, ok_ = oracle.bf_search_sq8(x, None, None, a.metric, qh[i], a.k)
            else:
                os_, ok_ = oracle.bf_search(x, None, a.metric, qh[i], a.k)
            ok &= bool(np.array_equal(lab[i], ok_) and np.array_equal(s[i].view(np.uint32), os_.view(np.uint32)))
        cpu = None
        if a.cpu_seconds > 0 and not a.quant:  # CPU baseline leg (BruteForceVectorIndex.Search per query)
            from bench import host_cpus
            host = host_cpus()
            th = host["usable"]
            S = min(a.nq, 4 * th)
            t = time.perf_counter()
            oracle.bf_search_batch(qh[:S], a.k, x, metric=a.metric, nthreads=th)
            S = int(min(a.nq, max(S, S * a.cpu_seconds / max(time.perf_counter() - t, 1e-3))))
            t = time.perf_counter()
            cs, ck, _ = oracle.bf_search_batch(qh[:S], a.k, x, metric=a.metric, nthreads=th)
            ct = time.perf_counter() - t
            cpu = {"value": S / ct, "unit": "queries/s", "cores": th, "kind": "port", "host": host,
                   "sample": f"{S} of the {a.nq} queries (oracle/oracle.c BruteForce search, one query per thread)",
                   "parity": {"queries": S, "ids_equal": bool(np.array_equal(ck, lab[:S])),
                              "scores_bit_identical": bool(np.array_equal(cs.view(np.uint32), s[:S].view(np.uint32)))}}
            log(f"cpu baseline {S / ct:,.1f} QPS on {th} threads")
        scan = phases.get("flat_scan", {"ms": float("nan"), "work": 0})
        out = {"workload": f"FLAT{' SQ8' if a.quant else ''} d={d} N={n} Q={a.nq} k={a.k} "
                           f"metric={['L2', 'IP', 'COS'][a.metric]}",
               "qps": qps, "ms_per_step": ms, "phases_ms": {k_: v["ms"] for k_, v in phases.items()},
               "scan_pairs": scan["work"],
               "scan_tflops_2d": scan["work"] * 2 * d / (scan["ms"] * 1e-3) / 1e12,
               # (query, row) pairs per second over the whole step; not a memory rate (the scan reads each
               # fp16 tile once per item of up to 512 queries, not once per query)
               "pairs_per_s": qps * n,
               "parity_sample": {"queries": a.check, "ids_and_bits_equal": ok}, "cpu_baseline": cpu}
    else:
        n, d = a.n or 3_200_000, a.dim or 768
        from pyrope_amd import generate_synthetic_blocked
        qh = generate_synthetic(a.nq, d, 1337)
        t = time.time()
        if a.train_rows > 0 and a.train_rows < n:
            # P1 at full size: train the coarse quantizer and the codebooks on the first train_rows rows
            # (reference-identical training on that sample), then stream every row into an index that
            # only assigns and encodes (set_centroids + set_codebooks, IvfPqIndex::build_given)
            xs = generate_synthetic_blocked(0, a.train_rows, d, 42)
            tr = IvfPqVectorIndex(d, a.metric, m=a.m, k=256, n_list=a.nlist)
            tr.add_labels(np.arange(a.train_rows, dtype=np.int64), xs, track_ids=False)
            tr.build()
            cents = tr.centroids_array()
            cb0 = tr.pq_state()[0]
            tr.close()
            del xs
            log(f"trained quantizers on {a.train_rows} rows in {time.time() - t:.1f}s")
            idx = IvfPqVectorIndex(d, a.metric, m=a.m, k=256, n_list=a.nlist)
            idx.set_centroids(cents)
            idx.set_codebooks(cb0)
            idx.reserve(n)
            step_rows = 1 << 20
            for r0 in range(0, n, step_rows):
                cn = min(step_rows, n - r0)
                idx.add_labels(np.arange(r0, r0 + cn, dtype=np.int64), generate_synthetic_blocked(r0, cn, d, 42),
                               track_ids=False)
                if (r0 // step_rows) % 8 == 0:
                    log(f"added {r0 + cn} rows ({time.time() - t:.1f}s)")
            x = None
        else:
            x = generate_synthetic(n, d, 42)
            idx = IvfPqVectorIndex(d, a.metric, m=a.m, k=256, n_list=a.nlist)
            idx.add_labels(np.arange(n, dtype=np.int64), x)
        idx.build()
        log(f"built IVF_PQ n={n} d={d} nlist={a.nlist} m={a.m} in {time.time() - t:.1f}s")
        q = torch.from_numpy(qh).cuda()
        opts = SearchOptions(nprobe=a.nprobe)
        qps, ms, phases, s, lab = timed(idx, q, a.nq, a.k, opts, a.steps, a.warmup, L)
        run_sweep(idx, q, opts, s, lab)
        cb, codes, off, labels, live = idx.pq_state()
        cents = idx.centroids_array()
        from concurrent.futures import ThreadPoolExecutor
        from bench import host_cpus
        chk = np.linspace(0, a.nq - 1, a.check).astype(int)

        def chk_one(i):  # the oracle's IvfPq search of query i (one query per thread; ctypes drops the GIL)
            os_, ok_ = oracle.ivfpq_search(qh[i], a.k, cents, codes, off, cb, live, metric=a.metric, nprobe=a.nprobe)
            return bool(np.array_equal(lab[i], labels[ok_]) and np.array_equal(s[i].view(np.uint32),
                                                                                 os_.view(np.uint32)))
        t1 = time.time()
        with ThreadPoolExecutor(host_cpus()["usable"]) as ex:
            eq = list(ex.map(chk_one, chk))
        ok = all(eq)
        log(f"parity: {sum(eq)} of {len(eq)} sampled queries bit-identical to the oracle ({time.time() - t1:.1f}s)")
        recall = None
        if a.recall_queries > 0:
            # recall@10 against the exact top-10 over all N rows: the base rows streamed through a FLAT L2
            # index chunk by chunk (BruteForceVectorIndex.Search, exact), per-query top-10 merged on the host
            R = min(a.recall_queries, a.nq)
            t1 = time.time()
            gs = np.full((R, a.k * 2), -np.inf, np.float32)
            gl = np.full((R, a.k * 2), -1, np.int64)
            step = 4 << 20
            for r0 in range(0, n, step):
                cn = min(step, n - r0)
                f = BruteForceVectorIndex(d, 0)
                f.add_labels(np.arange(r0, r0 + cn, dtype=np.int64), generate_synthetic_blocked(r0, cn, d, 42),
                             track_ids=False)
                fs, fl, _ = f.search_batch(qh[:R], a.k)
                f.close()
                log(f"recall truth: rows [{r0}, {r0 + cn}) ({time.time() - t1:.1f}s)")
                cs_, cl_ = np.concatenate([gs[:, :a.k], fs], 1), np.concatenate([gl[:, :a.k], fl], 1)
                o = np.lexsort((cl_, -cs_), axis=1)[:, :a.k]
                gs[:, :a.k], gl[:, :a.k] = np.take_along_axis(cs_, o, 1), np.take_along_axis(cl_, o, 1)
            gt = gl[:, :a.k]
            recall = sum(len(set(gt[i].tolist()) & set(lab[i].tolist())) for i in range(R)) / (R * a.k)
            log(f"recall@{a.k} over {R} queries: {recall:.4f} ({time.time() - t1:.1f}s)")
        cpu = None
        if a.cpu_seconds > 0:  # CPU baseline leg: the oracle's IvfPq search, one query per thread
            host = host_cpus()
            th = host["usable"]

            def one(i):
                return oracle.ivfpq_search(qh[i], a.k, cents, codes, off, cb, live, metric=a.metric, nprobe=a.nprobe)
            S = th
            with ThreadPoolExecutor(th) as ex:
                t1 = time.perf_counter()
                list(ex.map(one, range(S)))
                S = int(min(a.nq, max(S, S * a.cpu_seconds / max(time.perf_counter() - t1, 1e-3))))
                t1 = time.perf_counter()
                res = list(ex.map(one, range(S)))
                ct = time.perf_counter() - t1
            ids_eq = all(np.array_equal(lab[i], labels[r[1]]) for i, r in enumerate(res))
            bits_eq = all(np.array_equal(s[i].view(np.uint32), r[0].view(np.uint32)) for i, r in enumerate(res))
            cpu = {"value": S / ct, "unit": "queries/s", "cores": th, "kind": "port", "host": host,
                   "sample": f"{S} of the {a.nq} queries (oracle/oracle.c IvfPq search, one query per thread)",
                   "parity": {"queries": S, "ids_equal": bool(ids_eq), "scores_bit_identical": bool(bits_eq)}}
            log(f"cpu baseline {S / ct:,.1f} QPS on {th} threads")
        scan = phases.get("pq_scan", {"ms": float("nan"), "work": 0})
        out = {"workload": f"IVF_PQ d={d} N={n} nlist={a.nlist} m={a.m} k=256 nprobe={a.nprobe} Q={a.nq}",
               "training": (f"coarse k-means + codebooks trained (reference-identical) on the first {a.train_rows} "
                            f"rows, every row assigned + encoded" if 0 < a.train_rows < n else "all rows"),
               "qps": qps, "ms_per_step": ms, "phases_ms": {k_: v["ms"] for k_, v in phases.items()},
               "scan_rows": scan["work"],
               "lookups_per_s": scan["work"] * a.m / (scan["ms"] * 1e-3),
               "roofline": pq_roofline(scan["work"] * a.m / (scan["ms"] * 1e-3)),
               "parity_sample": {"queries": a.check, "ids_and_bits_equal": ok}, "recall_at_10": recall,
               "cpu_baseline": cpu}
        if os.environ.get("PYR_PQ_MFMA", "1") != "0" and "pq_scan" in phases:  # the matrix-core scan (pq32.hip)
            sc = phases["pq_scan"]
            tf = sc["work"] * 2 * d / (sc["ms"] * 1e-3) / 1e12
            out["lut_equiv"] = out.pop("roofline")  # what the LUT scan would need for the same rate
            out["roofline"] = {"bound": "mfma", "achieved": tf, "peak": 2500.0, "unit": "TFLOP/s", "frac": tf / 2500.0,
                               "note": "decoded (query, code row) pairs x 2 D fp16 MFMA flops over the scan phase "
                                       "(sample + main pass) vs the dense fp16 peak"}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
