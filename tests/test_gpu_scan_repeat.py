"""The list scan's answers must not depend on how its waves interleave (scan.hip).

Round 6 moved the fetch of a block's next work item ahead of the end-of-item barrier and, with it, the barrier
that separated an item's candidate flush from the next item's prologue: a wave that ran ahead rewrote the query
slot tables a slower wave's flush was still reading, and candidates landed in the wrong queries' buffers -- rarely
at N = 1, on most steps of the N = 8 rank shape.  These tests make the flush long (many emitted rows per item:
a low fixed sample rank, 512-query items over long lists) and repeat the same search, against the exact path.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


class _env:
    def __init__(self, **kv):
        self.kv = {k: str(v) for k, v in kv.items()}

    def __enter__(self):
        import os
        self.old = {k: os.environ.get(k) for k in self.kv}
        os.environ.update(self.kv)

    def __exit__(self, *a):
        import os
        for k, v in self.old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def _same(a, b):
    (s1, l1, c1), (s2, l2, c2) = a, b
    np.testing.assert_array_equal(l2, l1)
    assert np.array_equal(s2.view(np.uint32), s1.view(np.uint32))
    np.testing.assert_array_equal(c2, c1)


@pytest.mark.parametrize("metric", [0, 1])
def test_stream_scan_repeatable_under_heavy_emission(hiplib, metric):
    from pyrope_amd import IvfFlatVectorIndex, SearchOptions, generate_synthetic
    data = generate_synthetic(300_000, 64, 3)
    idx = IvfFlatVectorIndex(64, metric, n_list=48)
    idx.add_labels(np.arange(len(data), dtype=np.int64), data, track_ids=False)
    idx.build()
    q = generate_synthetic(8192, 64, 4)
    opts = SearchOptions(nprobe=8)
    with _env(PYR_FILTER=0):
        ref = idx.search_batch(q, 10, opts)
    for rank in (None, 48):  # the default sample rank, then a low threshold: ~10x the emitted rows
        env = {} if rank is None else {"PYR_STREAM_RANK": rank}
        with _env(**env):
            for _ in range(3):
                _same(ref, idx.search_batch(q, 10, opts))
