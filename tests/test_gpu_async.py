"""pyr_index_search_device is asynchronous (include/pyrope_ann.h: "Does not synchronize
the stream"): the IVF stream-and-emit search, its certificates and the exact re-run of certificate
failures are all enqueued on the caller's stream with device-side counts, so

- two batches enqueued back to back (no host synchronization between them) give each batch's own
  results, also when every certificate fails (PYR_FILTER_CERR: every query takes the device re-run);
- the search can be captured into a HIP graph and replayed with new queries in the same buffer.

Reference: Vector/IvfFlatVectorIndex.cs:147-231 (the search the results must equal)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


class _env:
    def __init__(self, **kv):
        self.kv = {k: str(v) for k, v in kv.items()}

    def __enter__(self):
        self.old = {k: os.environ.get(k) for k in self.kv}
        os.environ.update(self.kv)

    def __exit__(self, *a):
        for k, v in self.old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


_IDX = {}


def _index():
    from pyrope_amd import IvfFlatVectorIndex, generate_synthetic
    if "i" not in _IDX:
        x = generate_synthetic(120_000, 128, 42)
        idx = IvfFlatVectorIndex(128, 0, n_list=64)
        idx.add_labels(np.arange(len(x), dtype=np.int64), x)
        idx.build()
        _IDX["i"] = idx
    return _IDX["i"]


def _dev_search(idx, q, k, opts, stream):
    import torch
    s = torch.empty((q.shape[0], k), dtype=torch.float32, device="cuda")
    lab = torch.empty((q.shape[0], k), dtype=torch.int64, device="cuda")
    c = torch.empty((q.shape[0],), dtype=torch.int32, device="cuda")
    idx.search_device(q.data_ptr(), q.shape[0], k, s.data_ptr(), lab.data_ptr(), c.data_ptr(), stream.cuda_stream,
                      opts)
    return s, lab, c


def _same(dev, ref):
    s, lab, c = (t.cpu().numpy() for t in dev)
    np.testing.assert_array_equal(c, ref[2])
    np.testing.assert_array_equal(lab, ref[1])
    assert np.array_equal(s.view(np.uint32), ref[0].view(np.uint32))


@pytest.mark.parametrize("force_fail", [False, True])
def test_back_to_back_batches_without_host_sync(hiplib, force_fail):
    import torch

    from pyrope_amd import SearchOptions, generate_synthetic
    idx = _index()
    opts = SearchOptions(nprobe=16)
    qa, qb = generate_synthetic(700, 128, 1), generate_synthetic(500, 128, 2)
    env = {"PYR_FILTER_CERR": "1e15"} if force_fail else {}
    with _env(**env):
        ra, rb = idx.search_batch(qa, 10, opts), idx.search_batch(qb, 10, opts)
        st = torch.cuda.Stream()
        with torch.cuda.stream(st):
            da, db = torch.from_numpy(qa).cuda(), torch.from_numpy(qb).cuda()
            out_a = _dev_search(idx, da, 10, opts, st)
            out_b = _dev_search(idx, db, 10, opts, st)
        st.synchronize()
    with _env(PYR_FILTER=0):
        exact = idx.search_batch(qa, 10, opts)
    _same(out_a, ra)
    _same(out_b, rb)
    _same(out_a, exact)


def test_search_device_graph_capture_and_replay(hiplib):
    import torch

    from pyrope_amd import SearchOptions, generate_synthetic
    idx = _index()
    opts = SearchOptions(nprobe=16)
    n = 600
    qa, qb = generate_synthetic(n, 128, 3), generate_synthetic(n, 128, 4)
    ra, rb = idx.search_batch(qa, 10, opts), idx.search_batch(qb, 10, opts)
    st = torch.cuda.Stream()
    qbuf = torch.from_numpy(qa).cuda()
    with torch.cuda.stream(st):
        out = _dev_search(idx, qbuf, 10, opts, st)  # warm-up: the stream's workspace is sized
    st.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=st):
        idx.search_device(qbuf.data_ptr(), n, 10, out[0].data_ptr(), out[1].data_ptr(), out[2].data_ptr(),
                          st.cuda_stream, opts)
    qbuf.copy_(torch.from_numpy(qb))
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    _same(out, rb)
    qbuf.copy_(torch.from_numpy(qa))
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    _same(out, ra)


@pytest.mark.parametrize("nq", [1, 3, 40])
def test_device_rerun_chunks_long_lists(hiplib, nq):
    """A few failing queries split every probed list into up to 64 row chunks (kernels.hip
    ivf_rerun_scan_kernel: units (query, probe, chunk), then a merge over nprobe x chunks partial
    lists): long ragged lists (4 lists over 50,001 rows, some rows deleted) give the exact results."""
    from pyrope_amd import IvfFlatVectorIndex, SearchOptions, generate_synthetic
    x = generate_synthetic(50_001, 128, 7)
    idx = IvfFlatVectorIndex(128, 0, n_list=4)
    idx.add_labels(np.arange(len(x), dtype=np.int64), x)
    idx.build()
    for lab in range(0, 50_001, 97):
        assert idx.delete(str(lab))
    q = generate_synthetic(nq, 128, 8)
    opts = SearchOptions(nprobe=3)
    with _env(PYR_FILTER=0):
        exact = idx.search_batch(q, 10, opts)
    with _env(PYR_FILTER_CERR="1e15"):
        got = idx.search_batch(q, 10, opts)
    np.testing.assert_array_equal(got[2], exact[2])
    np.testing.assert_array_equal(got[1], exact[1])
    assert np.array_equal(got[0].view(np.uint32), exact[0].view(np.uint32))


_FLAT = {}


def _flat_index(metric):
    from pyrope_amd import BruteForceVectorIndex, generate_synthetic
    if metric not in _FLAT:
        x = generate_synthetic(60_000, 128, 42)
        idx = BruteForceVectorIndex(128, metric)
        idx.add_labels(np.arange(len(x), dtype=np.int64), x)
        _FLAT[metric] = idx
    return _FLAT[metric]


@pytest.mark.parametrize("force_fail", [False, True])
@pytest.mark.parametrize("metric", [0, 1, 2])
def test_flat_search_device_graph_capture_and_replay(hiplib, metric, force_fail):
    """FLAT search_device on the stream scan (L2, IP and Cosine) enqueues only -- the
    certificates and the exact re-run of failures run from device-side counts -- so it captures into a
    HIP graph (a host synchronization inside the capture would fail it); the graph, replayed with other
    queries in the captured buffer, returns their results, also when every certificate fails
    (PYR_FILTER_CERR: every query takes the device re-run).  Then two batches enqueued back to back on
    one stream without a host synchronization give each batch's own results."""
    import torch

    from pyrope_amd import generate_synthetic
    idx = _flat_index(metric)
    n = 300
    qa, qb = generate_synthetic(n, 128, 3), generate_synthetic(n, 128, 4)
    env = {"PYR_FILTER_CERR": "1e15"} if force_fail else {}
    with _env(**env):
        ra, rb = idx.search_batch(qa, 10), idx.search_batch(qb, 10)
        st = torch.cuda.Stream()
        qbuf = torch.from_numpy(qa).cuda()
        with torch.cuda.stream(st):
            out = _dev_search(idx, qbuf, 10, None, st)  # warm-up: workspace and row terms sized
        st.synchronize()
        if os.environ.get("PYR_DEBUG_ALLOC"):  # diagnostics: the caller's buffers beside the library's log
            with open(os.environ["PYR_DEBUG_ALLOC"], "a") as f:
                f.write(f"# test metric={metric} force_fail={force_fail} stream={st.cuda_stream:#x} "
                        f"qbuf={qbuf.data_ptr():#x} out={[hex(t.data_ptr()) for t in out]}\n")
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=st):
            idx.search_device(qbuf.data_ptr(), n, 10, out[0].data_ptr(), out[1].data_ptr(), out[2].data_ptr(),
                              st.cuda_stream, None)
        # replayed twice with other queries in the captured buffer (a search must be repeatable:
        # BruteForceVectorIndex.cs:275-379)
        for qv, ref in ((qb, rb), (qa, ra)):
            qbuf.copy_(torch.from_numpy(qv))
            torch.cuda.synchronize()
            g.replay()
            torch.cuda.synchronize()
            _same(out, ref)
        # back to back on the capture stream, no host synchronization in between ...
        qa_d, qb_d = torch.from_numpy(qa).cuda(), torch.from_numpy(qb).cuda()
        torch.cuda.synchronize()
        with torch.cuda.stream(st):
            oa = _dev_search(idx, qa_d, 10, None, st)
            ob = _dev_search(idx, qb_d, 10, None, st)
        st.synchronize()
        _same(oa, ra)
        _same(ob, rb)
        # ... and the graph replayed once more after those plain searches on its stream's workspace
        qbuf.copy_(torch.from_numpy(qb))
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        _same(out, rb)
    with _env(PYR_FILTER=0):
        _same(oa, idx.search_batch(qa, 10))
