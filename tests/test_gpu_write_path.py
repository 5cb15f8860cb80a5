"""The row-at-a-time write path: RowStore::write's small-batch path (one pinned staging copy +
one fused kernel, no host synchronization; engine.cpp, kernels.hip write_small_kernel), the searches that
must see those writes (Index::order_after_writes), the FLAT L2 tiles' center following the rows
(RowStore::recenter) and the re-encode when a row raises the fp16 scale.  Every answer is compared with the
bulk path (PYR_SMALL_WRITE=0) and the CPU oracle (BruteForceVectorIndex.cs:133-222, :275-379)."""
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


def _ops(seed, n, d):
    """a VEC.ADD-style stream: single rows, small batches, upserts of earlier ids, deletes"""
    rng = np.random.default_rng(seed)
    x = rng.standard_normal((n, d)).astype(np.float32)
    ops, i = [], 0
    while i < n:
        c = int(rng.choice([1, 1, 1, 3, 7, 64]))
        c = min(c, n - i)
        ops.append(("add", np.arange(i, i + c), x[i:i + c]))
        i += c
        if rng.random() < 0.1 and i > 10:
            j = rng.integers(0, i, 2)
            ops.append(("upsert", j, rng.standard_normal((2, d)).astype(np.float32)))
        if rng.random() < 0.05 and i > 10:
            ops.append(("delete", int(rng.integers(0, i)), None))
    return ops


def _apply(idx, ops, rows):
    for kind, lab, v in ops:
        if kind == "add":
            idx.add_labels(lab.astype(np.int64), v)
            rows.update({int(l): v[j] for j, l in enumerate(lab)})
        elif kind == "upsert":
            idx.upsert_batch([str(int(l)) for l in lab], v)
            rows.update({int(l): v[j] for j, l in enumerate(lab)})  # (the last of a repeated id wins)
        else:
            idx.delete(str(lab))
            rows.pop(lab, None)


@pytest.mark.parametrize("metric", [0, 1, 2])
@pytest.mark.parametrize("d", [64, 128])
def test_small_writes_equal_bulk_path_and_oracle(hiplib, oracle, metric, d):
    from pyrope_amd import BruteForceVectorIndex, generate_synthetic
    ops = _ops(3, 3000, d)
    q = generate_synthetic(24, d, 9)
    got, ref = [], []
    rows = {}
    for env, out in (({}, got), ({"PYR_SMALL_WRITE": 0}, ref)):
        with _env(**env):
            idx = BruteForceVectorIndex(d, metric)
            rows = {}
            for c in range(0, len(ops), 97):  # searches interleaved with the writes
                _apply(idx, ops[c:c + 97], rows)
                out.append(idx.search_batch(q, 10))
            idx.close()
    for a, b in zip(got, ref):
        np.testing.assert_array_equal(a[1], b[1])
        assert np.array_equal(a[0].view(np.uint32), b[0].view(np.uint32))
    # the final state against the oracle (live rows in slot order = label order here: ids never reused)
    labs = np.array(sorted(rows), np.int64)
    x = np.stack([rows[int(l)] for l in labs])
    s, l, _ = got[-1]
    for i in range(len(q)):
        os_, ok = oracle.bf_search(x, np.ones(len(x), np.uint8), metric, q[i], 10)
        np.testing.assert_array_equal(l[i][: len(ok)], labs[ok])
        assert np.array_equal(s[i][: len(os_)].view(np.uint32), os_.view(np.uint32))


def test_search_on_another_stream_sees_the_last_write(hiplib):
    """a small write returns before the device ran it: a device search on a different stream, issued right
    after, must still find the row (the stream waits for the write event)"""
    import torch

    from pyrope_amd import BruteForceVectorIndex, generate_synthetic
    d = 128
    idx = BruteForceVectorIndex(d, 0)
    idx.add_labels(np.arange(50_000, dtype=np.int64), generate_synthetic(50_000, d, 1), track_ids=False)
    q = torch.from_numpy(generate_synthetic(1, d, 2)).cuda()
    s = torch.empty((1, 1), dtype=torch.float32, device="cuda")
    lab = torch.empty((1, 1), dtype=torch.int64, device="cuda")
    st = torch.cuda.Stream()
    qh = q.cpu().numpy()
    for i in range(20):
        row = qh + np.float32(1e-3 * (20 - i))  # each new row is the nearest so far
        idx.add_labels(np.array([100_000 + i], np.int64), row, track_ids=False)
        idx.search_device(q.data_ptr(), 1, 1, s.data_ptr(), lab.data_ptr(), 0, st.cuda_stream)
        st.synchronize()
        assert int(lab[0, 0]) == 100_000 + i
    idx.close()


def test_scale_growth_and_recentring(hiplib, oracle):
    """a head whose first write is one row: its tiles are centred on that row until the store doubles
    (re-centred on the live rows each time, and at build); a row 10^4 x larger than any before raises the
    fp16 scale (the bulk path re-encodes every slot).  Answers stay the oracle's throughout."""
    from pyrope_amd import BruteForceVectorIndex, generate_synthetic
    d = 128
    x = generate_synthetic(5000, d, 4)
    x[3000] *= 1e4
    q = generate_synthetic(16, d, 5)
    idx = BruteForceVectorIndex(d, 0)
    idx.add_labels(np.arange(1, dtype=np.int64), x[:1])
    for i in range(1, 5000, 5):
        idx.add_labels(np.arange(i, min(5000, i + 5), dtype=np.int64), x[i:i + 5])
        if i % 1000 == 1:
            s, l, _ = idx.search_batch(q, 10)
            n = min(5000, i + 5)
            for j in range(0, 16, 5):
                os_, ok = oracle.bf_search(x[:n], np.ones(n, np.uint8), 0, q[j], 10)
                np.testing.assert_array_equal(l[j][: len(ok)], ok)
                assert np.array_equal(s[j][: len(os_)].view(np.uint32), os_.view(np.uint32))
    idx.build()  # re-centres on the live rows
    s, l, _ = idx.search_batch(q, 10)
    for j in range(16):
        os_, ok = oracle.bf_search(x, np.ones(5000, np.uint8), 0, q[j], 10)
        np.testing.assert_array_equal(l[j][: len(ok)], ok)
        assert np.array_equal(s[j][: len(os_)].view(np.uint32), os_.view(np.uint32))
    idx.close()
