"""pyrope_amd -- MI355X (gfx950) engine for Pyrope's batched ANN distance-scan path.

The product is libpyrope_hip.so (HIP kernels + C ABI, include/pyrope_ann.h);
this package holds its in-tree build script, the ctypes binding and the host
mirror of the reference's IVectorIndex plugin surface.
"""
from .vector import (BruteForceVectorIndex, DeltaVectorIndex, HipVectorIndex, ICentroidsProvider,  # noqa: F401
                     IndexStats, IvfFlatVectorIndex, IvfPqVectorIndex, IVectorIndex, ScalarQuantizer, SearchOptions,
                     SearchResult, VectorIndexRegistry, VectorMetric, generate_synthetic,
                     generate_synthetic_blocked, kmeans_train, assign)
from ._lib import (ArgumentException, ArgumentNullException, ArgumentOutOfRangeException,  # noqa: F401
                   DeviceError, InvalidOperationException)

__version__ = "0.1.0"
