"""GPU k-means (KMeansUtils.Train, KMeansUtils.cs:10-68) is bit-identical to the oracle's."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("metric,dim,n,k", [(0, 128, 5000, 50), (1, 64, 3000, 17), (2, 128, 4000, 33),
                                            (0, 8, 2000, 256), (0, 3, 500, 7), (0, 128, 40, 100)])
def test_kmeans_via_build(hiplib, oracle, metric, dim, n, k):
    from pyrope_amd import IvfFlatVectorIndex, generate_synthetic
    x = generate_synthetic(n, dim, 11)
    idx = IvfFlatVectorIndex(dim, metric, n_list=k)
    idx.add_labels(np.arange(n), x)
    idx.build()
    cents = oracle.kmeans_train(x, k, metric, 10, 42)
    g = idx.centroids_array()
    assert g.shape == cents.shape
    assert np.array_equal(g.view(np.uint32), cents.view(np.uint32))
