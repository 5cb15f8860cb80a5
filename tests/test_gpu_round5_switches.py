"""Round-5 kernels against their A/B switches: every switch must leave the answers bit-identical.

  PYR_SAMPLE16=1      the sample pass on sample16_kernel instead of the scan kernel's SMP mode (scan.hip)
  PYR_SPREP_Q=0       list-major query operands instead of sprep_q_kernel (sample16.hip)
  PYR_RERUN_FUSED=0   the exact re-run's separate merge launch instead of the last unit's merge (kernels.hip)
  PYR_FILTER_ABLATE=1024 / 2048   round 4's B-operand schedule / the emission without 4-row block tests

T_q may change in its last bits with the sample kernel (its values group rows differently), which changes the
emitted rows, never the certified answers (IvfFlatVectorIndex.cs:147-231, BruteForceVectorIndex.cs:275-379).
"""
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


def _same(a, b):
    np.testing.assert_array_equal(a[1], b[1])
    assert np.array_equal(a[0].view(np.uint32), b[0].view(np.uint32))


SWITCHES = [{"PYR_SAMPLE16": 1}, {"PYR_SPREP_Q": 0}, {"PYR_FILTER_ABLATE": 1024}, {"PYR_FILTER_ABLATE": 2048}]


@pytest.mark.parametrize("metric", [0, 1])
def test_ivf_switches_same_answers(hiplib, oracle, metric):
    from pyrope_amd import IvfFlatVectorIndex, SearchOptions, assign, generate_synthetic
    d, n = 128, 30000
    x = generate_synthetic(n, d, 21)
    idx = IvfFlatVectorIndex(d, metric, n_list=24)
    idx.add_labels(np.arange(n, dtype=np.int64), x, track_ids=False)
    idx.build()
    q = generate_synthetic(700, d, 22)
    opts = SearchOptions(nprobe=5)
    ref = idx.search_batch(q, 10, opts)
    for sw in SWITCHES:
        with _env(**sw):
            _same(idx.search_batch(q, 10, opts), ref)
    # the exact re-run: every certificate forced to fail, fused merge vs separate
    with _env(PYR_FILTER_CERR="1e15"):
        fused = idx.search_batch(q, 10, opts)
        with _env(PYR_RERUN_FUSED=0):
            sep = idx.search_batch(q, 10, opts)
    _same(fused, ref)
    _same(sep, ref)
    cents = idx.centroids_array()
    a = np.asarray(assign(cents, x, 0)) if metric == 0 else None  # the index's own (reference) assignment
    if a is not None:  # a few answers against the oracle (rows in list order, label order inside a list)
        order = np.argsort(a, kind="stable")
        off = np.concatenate([[0], np.cumsum(np.bincount(a, minlength=len(cents)))]).astype(np.int64)
        for i in range(0, len(q), 173):
            os_, ok = oracle.ivf_search(q[i], 10, cents, x[order], off, metric=0, nprobe=5)
            np.testing.assert_array_equal(ref[1][i][: len(ok)], order[ok])
            assert np.array_equal(ref[0][i][: len(os_)].view(np.uint32), os_.view(np.uint32))
    idx.close()


@pytest.mark.parametrize("metric", [0, 1, 2])
def test_flat_switches_same_answers(hiplib, metric):
    from pyrope_amd import BruteForceVectorIndex, generate_synthetic
    d, n = 128, 40000
    idx = BruteForceVectorIndex(d, metric)
    idx.add_labels(np.arange(n, dtype=np.int64), generate_synthetic(n, d, 31), track_ids=False)
    q = generate_synthetic(300, d, 32)
    ref = idx.search_batch(q, 10)
    for sw in SWITCHES:
        with _env(**sw):
            _same(idx.search_batch(q, 10), ref)
    idx.close()
