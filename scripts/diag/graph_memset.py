"""Do hipMemsetAsync nodes of a captured HIP graph clear their buffer on EVERY replay? (diagnostic)

The FLAT search faulted on the second replay of a captured graph while the IVF search,
the same kernels with larger work-list buffers, did not.  The search resets its counters with
hipMemsetAsync (the per-list counts of the work lists: 4 x nlist bytes -- 44 bytes for a FLAT store of
11 chunks, 256 for the IVF test's 64 lists).  This captures, per size, `memset(buf, 0)` followed by a
kernel that adds 1 to every word, replays the graph 3 times and reads the buffer back: a memset node that
works leaves 1 everywhere; one that does not leaves 3.  No out-of-bounds access is possible.
"""
import ctypes as C
import sys


def main():
    import torch
    torch.cuda.init()
    hip = C.CDLL("libamdhip64.so.7")  # torch's runtime (already loaded, resolved by its soname)
    hip.hipMemsetAsync.argtypes = [C.c_void_p, C.c_int, C.c_size_t, C.c_void_p]
    hip.hipMemsetD32Async.argtypes = [C.c_void_p, C.c_int, C.c_size_t, C.c_void_p]
    ok_all = True
    for fn in ("hipMemsetAsync", "hipMemsetD32Async"):
        for words in (1, 2, 3, 4, 11, 12, 16, 33, 64, 300, 1024):
            buf = torch.zeros(words + 64, dtype=torch.int32, device="cuda")  # tail guard: must stay 0
            st = torch.cuda.Stream()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=st):
                if fn == "hipMemsetAsync":
                    rc = hip.hipMemsetAsync(C.c_void_p(buf.data_ptr()), 0, 4 * words, C.c_void_p(st.cuda_stream))
                else:
                    rc = hip.hipMemsetD32Async(C.c_void_p(buf.data_ptr()), 0, words, C.c_void_p(st.cuda_stream))
                buf[:words].add_(1)
            assert rc == 0, rc
            got = []
            for _ in range(3):
                g.replay()
                torch.cuda.synchronize()
                got.append(buf[:words].cpu().tolist())
            tail = buf[words:].cpu()
            ok = all(all(v == 1 for v in r) for r in got) and int(tail.abs().sum()) == 0
            ok_all &= ok
            print(f"{fn:18s} {words:5d} words: after replays {[sorted(set(r)) for r in got]} tail clean "
                  f"{int(tail.abs().sum()) == 0} -> {'ok' if ok else 'MEMSET NODE NOT APPLIED'}", flush=True)
    # device-to-device hipMemcpyAsync nodes: copy a source of 7s over the buffer, then add 1 (8 expected)
    hip.hipMemcpyAsync.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p]
    for words in (1, 11, 300):
        src = torch.full((words,), 7, dtype=torch.int32, device="cuda")
        buf = torch.zeros(words, dtype=torch.int32, device="cuda")
        st = torch.cuda.Stream()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=st):
            rc = hip.hipMemcpyAsync(C.c_void_p(buf.data_ptr()), C.c_void_p(src.data_ptr()), 4 * words, 3,
                                    C.c_void_p(st.cuda_stream))
            buf.add_(1)
        assert rc == 0, rc
        got = []
        for _ in range(3):
            g.replay()
            torch.cuda.synchronize()
            got.append(sorted(set(buf.cpu().tolist())))
        ok = all(r == [8] for r in got)
        ok_all &= ok
        print(f"hipMemcpyAsync D2D  {words:5d} words: after replays {got} -> {'ok' if ok else 'COPY NODE WRONG'}",
              flush=True)
    # the library's replacement (pyrope_amd WordFill kernel) is an ordinary kernel node: checked by
    # tests/test_gpu_async.py's FLAT graph test (replayed three times)
    print("all memset / memcpy nodes applied on every replay:", ok_all, flush=True)
    return 0 if ok_all else 1


if __name__ == "__main__":
    sys.exit(main())
