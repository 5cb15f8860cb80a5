"""The FLAT graph test's exact sequence (diagnostic): capture with qa, replay with qb, replay with qa;
markers on stderr so that an AMD_LOG_LEVEL=3 log shows the kernels dispatched by each replay."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch
    torch.cuda.init()
    from pyrope_amd import BruteForceVectorIndex, generate_synthetic
    n = 300
    qa, qb = generate_synthetic(n, 128, 3), generate_synthetic(n, 128, 4)
    x = generate_synthetic(60_000, 128, 42)
    idx = BruteForceVectorIndex(128, 0)
    idx.add_labels(np.arange(len(x), dtype=np.int64), x)
    ra, rb = idx.search_batch(qa, 10), idx.search_batch(qb, 10)
    st = torch.cuda.Stream()
    qbuf = torch.from_numpy(qa).cuda()
    with torch.cuda.stream(st):
        s = torch.empty((n, 10), dtype=torch.float32, device="cuda")
        lab = torch.empty((n, 10), dtype=torch.int64, device="cuda")
        c = torch.empty((n,), dtype=torch.int32, device="cuda")
        idx.search_device(qbuf.data_ptr(), n, 10, s.data_ptr(), lab.data_ptr(), c.data_ptr(), st.cuda_stream, None)
    st.synchronize()
    g = torch.cuda.CUDAGraph()
    print("### capture", file=sys.stderr, flush=True)
    with torch.cuda.graph(g, stream=st):
        idx.search_device(qbuf.data_ptr(), n, 10, s.data_ptr(), lab.data_ptr(), c.data_ptr(), st.cuda_stream, None)
    for name, qv, ref in (("qb", qb, rb), ("qa", qa, ra)):
        qbuf.copy_(torch.from_numpy(qv))
        torch.cuda.synchronize()
        print(f"### replay {name}", file=sys.stderr, flush=True)
        g.replay()
        torch.cuda.synchronize()
        print(f"replay {name}: equal {np.array_equal(lab.cpu().numpy(), ref[1])}", flush=True)


if __name__ == "__main__":
    main()
