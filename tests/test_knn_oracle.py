"""Pins the kNN oracle (oracle/knn_oracle.cpp, the simple_knn.cu restatement) to an
exact 3-nearest-neighbour search (scipy cKDTree in float64): the reference's box
pruning never drops a true neighbour, so both give the same mean squared distance
up to fp32 rounding of the distances."""
import numpy as np
import pytest
from scipy.spatial import cKDTree


@pytest.mark.parametrize("P,seed", [(4, 0), (50, 1), (1023, 2), (1025, 3), (20000, 4)])
def test_oracle_is_exact_knn(oracle_mod, P, seed):
    rng = np.random.default_rng(seed)
    pts = rng.uniform(-1.3, 1.3, (P, 3)).astype(np.float32)
    if P > 10:
        pts[P // 2] = pts[P // 3]
    got = oracle_mod.dist_knn3(pts)
    dd, _ = cKDTree(pts.astype(np.float64)).query(pts.astype(np.float64), k=4)
    ref = (dd[:, 1:] ** 2).mean(1)
    np.testing.assert_allclose(got, ref, rtol=1e-6, atol=1e-12)


def test_oracle_fewer_than_three_neighbours_is_inf(oracle_mod):
    # best[] keeps FLT_MAX entries: (FLT_MAX + FLT_MAX + d) / 3 overflows to inf, as on the GPU
    assert np.isinf(oracle_mod.dist_knn3(np.zeros((2, 3), np.float32))).all()
