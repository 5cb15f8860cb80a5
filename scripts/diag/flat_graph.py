"""Graph capture of FLAT search_device vs IVF (diagnostic, measurement only): node counts by type of the
captured HIP graph; with REPLAY=1 also replays it once with the captured queries and compares."""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

TYPES = {0: "kernel", 1: "memcpy", 2: "memset", 3: "host", 4: "graph", 5: "empty", 6: "wait_event",
         7: "event_record", 10: "mem_alloc", 11: "mem_free"}


def nodes(hip, graph):
    n = C.c_size_t(0)
    assert hip.hipGraphGetNodes(C.c_void_p(graph), None, C.byref(n)) == 0
    arr = (C.c_void_p * n.value)()
    assert hip.hipGraphGetNodes(C.c_void_p(graph), arr, C.byref(n)) == 0
    cnt = {}
    for i in range(n.value):
        t = C.c_int(-1)
        hip.hipGraphNodeGetType(C.c_void_p(arr[i]), C.byref(t))
        cnt[TYPES.get(t.value, t.value)] = cnt.get(TYPES.get(t.value, t.value), 0) + 1
    return cnt


def main():
    import torch
    torch.cuda.init()
    from pyrope_amd import BruteForceVectorIndex, IvfFlatVectorIndex, SearchOptions, generate_synthetic
    hip = C.CDLL("libamdhip64.so")
    n = 300
    qa = generate_synthetic(n, 128, 3)
    x = generate_synthetic(60_000, 128, 42)
    for kind in ("ivf", "flat"):
        if kind == "flat":
            idx = BruteForceVectorIndex(128, 0)
            opts = None
        else:
            idx = IvfFlatVectorIndex(128, 0, n_list=64)
            opts = SearchOptions(nprobe=16)
        idx.add_labels(np.arange(len(x), dtype=np.int64), x)
        if kind == "ivf":
            idx.build()
        ra = idx.search_batch(qa, 10, opts)
        st = torch.cuda.Stream()
        qbuf = torch.from_numpy(qa).cuda()
        s = torch.empty((n, 10), dtype=torch.float32, device="cuda")
        lab = torch.empty((n, 10), dtype=torch.int64, device="cuda")
        c = torch.empty((n,), dtype=torch.int32, device="cuda")
        idx.search_device(qbuf.data_ptr(), n, 10, s.data_ptr(), lab.data_ptr(), c.data_ptr(), st.cuda_stream, opts)
        st.synchronize()
        ok0 = np.array_equal(lab.cpu().numpy(), ra[1])
        g = torch.cuda.CUDAGraph(keep_graph=True)
        try:
            with torch.cuda.graph(g, stream=st):
                idx.search_device(qbuf.data_ptr(), n, 10, s.data_ptr(), lab.data_ptr(), c.data_ptr(), st.cuda_stream,
                                  opts)
        except Exception as e:  # noqa: BLE001
            print(f"{kind}: capture raised {type(e).__name__}: {e}", flush=True)
            continue
        print(f"{kind}: direct search equal {ok0}; captured nodes {nodes(hip, g.raw_cuda_graph())}", flush=True)
        if os.environ.get("REPLAY") == "1":
            s.zero_()
            torch.cuda.synchronize()
            g.instantiate()
            g.replay()
            torch.cuda.synchronize()
            print(f"{kind}: replay equal {np.array_equal(lab.cpu().numpy(), ra[1])}", flush=True)


if __name__ == "__main__":
    main()
