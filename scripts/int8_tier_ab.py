"""8-bit residual tile tier vs the fp16 tiles at I1: how many rows each would emit (measurement).

The list scan emits every row whose upper bound reaches the query's sampled threshold T_q; the bound is the
filter's approximate score plus its error term.  An int8 tier (per-row or per-tile scale s, codes
round((x - c) / s) in [-127, 127], exact int32 dot products on v_mfma_i32_32x32x32_i8) halves the tile bytes
and the MFMA count, but its quantization error is far above fp16 rounding.  For the same T_q (the engine's,
read back from the rows it emitted: the lowest emitted bound) this script counts, per sampled query, the rows
of its probed lists whose int8 bound reaches T_q:

    approx = 2 s_q s_r sum(a_i b_i) - |x - c|^2 - |q - c|^2          (real arithmetic, a / b the int8 codes)
    |2 (q-c).(x-c) - 2 s_q s_r sum(a b)| <= s_q |x - c|_1 + s_r (|q - c|_1 + D s_q / 2)

(rounding to nearest: |e_q| <= s_q / 2, |e_x| <= s_r / 2 per dim), per-row scale and per-tile scale (32 rows
of a list share s_t and the largest |x - c|_1, what an epilogue of one fma per value allows).  The fp16 count
is the engine's own emission for the same queries (pyr_index_debug_candidates).  fp32 evaluation terms of
the int8 path are left out (they only add to its count).

    python scripts/int8_tier_ab.py [--n 10000000 --sample 200]
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
    ap.add_argument("--n", type=int, default=10_000_000)
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--nlist", type=int, default=1024)
    ap.add_argument("--nprobe", type=int, default=32)
    ap.add_argument("--nq", type=int, default=10_000)
    ap.add_argument("--sample", type=int, default=200)
    ap.add_argument("--cap", type=int, default=2048)
    args = ap.parse_args()
    import torch
    torch.cuda.init()
    from pyrope_amd import (IvfFlatVectorIndex, SearchOptions, _lib, assign, generate_synthetic,
                            generate_synthetic_blocked, kmeans_train)
    L = _lib.load()
    N, D, NL, P = args.n, args.dim, args.nlist, args.nprobe
    t = time.time()
    data = generate_synthetic_blocked(0, N, D, 42, 65536)
    cents = kmeans_train(data, NL, 0, 10, 42)
    a = np.concatenate([assign(cents, data[i:i + 2_000_000], 0) for i in range(0, N, 2_000_000)])
    idx = IvfFlatVectorIndex(D, 0, n_list=NL)
    idx.set_centroids(cents)
    idx.reserve(N)
    for i in range(0, N, 2_000_000):
        idx.add_labels(np.arange(i, min(N, i + 2_000_000), dtype=np.int64), data[i:i + 2_000_000], track_ids=False)
    idx.build()
    print(f"[int8] built I1 in {time.time() - t:.1f}s", flush=True)
    q = generate_synthetic(args.nq, D, 1337)
    idx.search_batch(q, 10, SearchOptions(nprobe=P))
    ub = np.empty((args.nq, args.cap), np.float32)
    lab = np.empty((args.nq, args.cap), np.int64)
    cnt = np.empty(args.nq, np.int32)
    rc = L.pyr_index_debug_candidates(idx._h, args.nq, args.cap, ub.ctypes.data_as(C.c_void_p),
                                      lab.ctypes.data_as(C.c_void_p), cnt.ctypes.data_as(C.c_void_p))
    assert rc == 0, L.pyr_last_error()
    idx.close()

    dev = torch.device("cuda", 0)
    X = torch.from_numpy(data).to(dev)
    Cn = torch.from_numpy(cents).to(dev)
    order = np.argsort(a, kind="stable")  # list-major, label order inside a list (the index's storage order)
    off = np.concatenate([[0], np.cumsum(np.bincount(a, minlength=NL))])
    order_d = torch.from_numpy(order).to(dev)
    inv = np.empty(N, np.int64)
    inv[order] = np.arange(N)
    rows16, rows8r, rows8t, hits16, hits8r, hits8t = [], [], [], [], [], []
    for i in range(min(args.sample, args.nq)):
        if cnt[i] <= 0 or cnt[i] > args.cap:
            continue
        T = float(ub[i, :cnt[i]].min())  # the engine's threshold, from above
        qv = torch.from_numpy(q[i]).to(dev)
        probes = torch.topk(-((Cn - qv) ** 2).sum(1), P).indices.cpu().numpy()
        n8r = n8t = 0
        t8r = t8t = 0
        for l in probes:
            sel = order_d[off[l]:off[l + 1]]
            if len(sel) == 0:
                continue
            R = X[sel] - Cn[l]                     # residual rows
            r = qv - Cn[l]
            sq = r.abs().max() / 127.0
            A = torch.round(r / sq)
            Q1 = r.abs().sum()
            x2 = (R * R).sum(1)
            r2 = (r * r).sum()
            X1 = R.abs().sum(1)
            # per-row scale
            s = R.abs().max(1).values / 127.0
            B = torch.round(R / s[:, None].clamp_min(1e-30))
            dot = (B.double() @ A.double()).float()
            u8 = 2 * sq * s * dot - x2 - r2 + sq * X1 + s * (Q1 + D * sq / 2)
            n8r += int((u8 >= T).sum())
            # per-tile scale: 32 consecutive rows of the list share s_t and max |x - c|_1
            nt = (len(sel) + 31) // 32
            pad = nt * 32 - len(sel)
            st = torch.nn.functional.pad(R.abs().max(1).values, (0, pad)).view(nt, 32).max(1).values / 127.0
            wt = torch.nn.functional.pad(X1, (0, pad)).view(nt, 32).max(1).values
            s_t = st.repeat_interleave(32)[:len(sel)]
            w_t = wt.repeat_interleave(32)[:len(sel)]
            Bt = torch.round(R / s_t[:, None].clamp_min(1e-30))
            dott = (Bt.double() @ A.double()).float()
            u8t = 2 * sq * s_t * dott - x2 - r2 + sq * w_t + s_t * (Q1 + D * sq / 2)
            m = (u8t >= T)
            n8t += int(m.sum())
            # tiles holding an emitted row (the per-(tile, group) emit branch is taken for such tiles)
            t8t += int(torch.nn.functional.pad(m.int(), (0, pad)).view(nt, 32).any(1).sum())
            t8r += int(torch.nn.functional.pad((u8 >= T).int(), (0, pad)).view(nt, 32).any(1).sum())
        rows16.append(int(cnt[i]))
        rows8r.append(n8r)
        rows8t.append(n8t)
        hits8r.append(t8r)
        hits8t.append(t8t)
        # the tiles the fp16 scan's emitted rows sit in
        li = lab[i, :cnt[i]]
        li = li[li >= 0]
        hits16.append(len(set(zip(a[li].tolist(), ((inv[li] - off[a[li]]) // 32).tolist()))))
    out = {"queries": len(rows16), "emitted_rows_per_query": {"fp16_engine": float(np.mean(rows16)),
                                                              "int8_per_row_scale": float(np.mean(rows8r)),
                                                              "int8_per_tile_scale": float(np.mean(rows8t))},
           "ratio_int8_row_over_fp16": float(np.mean(rows8r) / np.mean(rows16)),
           "ratio_int8_tile_over_fp16": float(np.mean(rows8t) / np.mean(rows16)),
           "emitting_tiles_per_query": {"fp16_engine": float(np.mean(hits16)),
                                        "int8_per_row_scale": float(np.mean(hits8r)),
                                        "int8_per_tile_scale": float(np.mean(hits8t))}}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
