"""Generates tests/golden/*.npz from the CPU oracle (oracle/oracle.c).

The reference (C#/.NET 8) cannot run in this image, so these fixtures pin the
restatement against itself over time and give the GPU tests an answer key that
does not depend on rebuilding the oracle.  Inputs are NOT stored: they are the
Pyrope.Benchmarks generator's output for the recorded seeds (Program.cs:251-263),
whose first values are stored as a pin of the generator itself.

    python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
import oracle as O  # noqa: E402


def main():
    out = {}
    # generator pins
    out["gen_seed42_first16"] = O.generate_vectors(2, 8, 42).reshape(-1)
    out["gen_seed1337_first16"] = O.generate_vectors(2, 8, 1337).reshape(-1)
    r = O.NetRandom(0)
    out["random_seed0_next5"] = np.array([r.next() for _ in range(5)], np.int64)
    np.savez_compressed(os.path.join(HERE, "generator.npz"), **out)

    # FLAT d=128 N=2048 Q=32 k=10, L2 / IP / Cosine (BruteForceVectorIndex.Search)
    x = O.generate_vectors(2048, 128, 42)
    q = O.generate_vectors(32, 128, 1337)
    flat = {"n": 2048, "dim": 128, "nq": 32, "k": 10, "base_seed": 42, "query_seed": 1337}
    for m, name in [(0, "l2"), (1, "ip"), (2, "cos")]:
        s = np.zeros((32, 10), np.float32)
        kk = np.zeros((32, 10), np.int64)
        for i in range(32):
            s[i], kk[i] = O.bf_search(x, None, m, q[i], 10)
        flat[f"{name}_scores"] = s
        flat[f"{name}_keys"] = kk
    np.savez_compressed(os.path.join(HERE, "flat_d128.npz"), **flat)

    # IVF-Flat N=8192 nlist=64 nprobe=8 (IvfFlatVectorIndex Build + Search), L2
    x = O.generate_vectors(8192, 128, 42)
    q = O.generate_vectors(32, 128, 1337)
    cents, assign = O.ivf_build(x, 64, 0)
    rows, order, off = O.lists_from_assign(x, assign, len(cents))
    s = np.zeros((32, 10), np.float32)
    kk = np.zeros((32, 10), np.int64)
    for i in range(32):
        s[i], kk[i] = O.ivf_search(q[i], 10, cents, rows, off, metric=0, nprobe=8)
    np.savez_compressed(os.path.join(HERE, "ivf_flat.npz"), n=8192, dim=128, nlist=64, nprobe=8, k=10,
                        centroids=cents, assign=assign, scores=s, labels=order[kk])

    # IVF-PQ d=64 m=8 K=256 N=8192 nlist=32 nprobe=4 (IvfPqVectorIndex Build + Search), L2
    x = O.generate_vectors(8192, 64, 42)
    q = O.generate_vectors(32, 64, 1337)
    cents, assign, cb, codes = O.ivfpq_build(x, 32, 8, 256, 0)
    _, order, off = O.lists_from_assign(x, assign, len(cents))
    lcodes = codes[order]
    s = np.zeros((32, 10), np.float32)
    kk = np.zeros((32, 10), np.int64)
    for i in range(32):
        s[i], kk[i] = O.ivfpq_search(q[i], 10, cents, lcodes, off, cb, nprobe=4)
    np.savez_compressed(os.path.join(HERE, "ivf_pq.npz"), n=8192, dim=64, nlist=32, m=8, ksub=256, nprobe=4, k=10,
                        centroids=cents, assign=assign, codebooks=cb, codes=codes, scores=s, labels=order[kk])
    print("wrote", sorted(f for f in os.listdir(HERE) if f.endswith(".npz")))


if __name__ == "__main__":
    main()
