"""FLAT (BruteForce) with k > 60 at the F2 shape (d = 128, N = 1M, 10,000 resident queries): the stream scan with
the deep refine vs the exact VALU scan (PYR_DEEP_REFINE=0), bit-identical answers required.

    python scripts/flat_deepk_ab.py [--n 1000000 --topk 100,200,256]
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--nq", type=int, default=10_000)
    ap.add_argument("--metric", type=int, default=0)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--topk", default="10,100,200,256")
    args = ap.parse_args()
    import torch
    torch.cuda.init()
    from pyrope_amd import BruteForceVectorIndex, generate_synthetic
    idx = BruteForceVectorIndex(args.dim, args.metric)
    for i in range(0, args.n, 500_000):
        m = min(500_000, args.n - i)
        idx.add_labels(np.arange(i, i + m, dtype=np.int64), generate_synthetic(m, args.dim, 1000 + i), track_ids=False)
    dev = torch.device("cuda", 0)
    q = torch.from_numpy(generate_synthetic(args.nq, args.dim, 1337)).to(dev)
    st = torch.cuda.current_stream()

    def run(k):
        s = torch.empty((args.nq, k), dtype=torch.float32, device=dev)
        lab = torch.empty((args.nq, k), dtype=torch.int64, device=dev)
        c = torch.empty(args.nq, dtype=torch.int32, device=dev)
        idx.search_device(q.data_ptr(), args.nq, k, s.data_ptr(), lab.data_ptr(), c.data_ptr(), stream=st.cuda_stream)
        return s, lab, c

    def timed(k):
        out = run(k)
        torch.cuda.synchronize()
        ts = []
        for _ in range(args.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            out = run(k)
            e1.record(st)
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        return float(np.median(ts)), [t.cpu().numpy() for t in out]

    res = {"config": {"n": args.n, "dim": args.dim, "nq": args.nq, "metric": args.metric}, "topk": {}}
    for k in [int(v) for v in args.topk.split(",") if v]:
        ms_s, out_s = timed(k)
        os.environ["PYR_DEEP_REFINE"] = "0"
        try:
            ms_e, out_e = timed(k)
        finally:
            os.environ.pop("PYR_DEEP_REFINE", None)
        os.environ["PYR_STREAM_DEBUG"] = "1"
        try:
            run(k)
            torch.cuda.synchronize()
        finally:
            os.environ.pop("PYR_STREAM_DEBUG", None)
        same = (np.array_equal(out_s[1], out_e[1]) and np.array_equal(out_s[2], out_e[2]) and
                np.array_equal(out_s[0].view(np.uint32), out_e[0].view(np.uint32)))
        res["topk"][str(k)] = {"stream_ms": ms_s, "exact_ms": ms_e, "speedup": ms_e / ms_s, "bit_identical": bool(same)}
        print(f"[flat deepk] k {k}: stream {ms_s:.3f} ms, exact {ms_e:.3f} ms, x{ms_e / ms_s:.1f}, identical {same}",
              flush=True)
    print(json.dumps(res), flush=True)
    idx.close()


if __name__ == "__main__":
    main()
