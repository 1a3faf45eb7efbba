"""distCUDA2 on the GPU against the CPU restatement of
simple_knn.cu (oracle/knn_oracle.cpp), itself checked against an exact kNN search
in tests/test_knn_oracle.py.  Tolerance: rtol 2e-6 (each squared distance is three
fp32 products and two adds; only contraction/ordering may differ), inf where the
reference yields inf (fewer than 3 other points)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _check(pts, oracle_mod):
    from gsr_train import distCUDA2
    got = distCUDA2(torch.from_numpy(pts).cuda()).cpu().numpy()
    ref = oracle_mod.dist_knn3(pts)
    fin = np.isfinite(ref)
    assert np.array_equal(fin, np.isfinite(got))
    np.testing.assert_allclose(got[fin], ref[fin], rtol=2e-6, atol=0)


@pytest.mark.parametrize("P", [1, 2, 3, 4, 5, 255, 256, 257, 1000, 65537])
def test_uniform(gpu_available, oracle_mod, P):
    rng = np.random.default_rng(P)
    _check(rng.uniform(-1.3, 1.3, (P, 3)).astype(np.float32), oracle_mod)


def test_duplicates_clusters_and_offsets(gpu_available, oracle_mod):
    rng = np.random.default_rng(7)
    centers = rng.uniform(5, 9, (20, 3))  # all points far from the origin (bounds include it)
    pts = (centers[rng.integers(0, 20, 30000)] + rng.normal(0, 0.01, (30000, 3))).astype(np.float32)
    pts[100:110] = pts[5]  # exact duplicates: distance 0 neighbours
    pts[200:205, 2] = 7.0  # a flat patch
    _check(pts, oracle_mod)


def test_degenerate_axis(gpu_available, oracle_mod):
    rng = np.random.default_rng(8)
    pts = rng.uniform(0, 1, (5000, 3)).astype(np.float32)
    pts[:, 1] = 0.0  # zero extent on y (0/0 in the Morton quantisation, as in the reference)
    _check(pts, oracle_mod)


def test_large_scene(gpu_available, oracle_mod):
    rng = np.random.default_rng(9)
    _check(rng.uniform(-1.5, 1.5, (400_000, 3)).astype(np.float32), oracle_mod)


def test_create_from_pcd(gpu_available, oracle_mod):
    from collections import namedtuple
    from gsr_train import GaussianModel
    Pcd = namedtuple("BasicPointCloud", ["points", "colors", "normals"])
    rng = np.random.default_rng(10)
    pts = rng.uniform(-1, 1, (3000, 3)).astype(np.float32)
    cols = rng.uniform(0, 1, (3000, 3)).astype(np.float32)
    m = GaussianModel(3, device="cuda")
    m.create_from_pcd(Pcd(pts, cols, np.zeros_like(pts)), 2.5)
    assert m.spatial_lr_scale == 2.5 and m.num_points == 3000
    d2 = np.maximum(oracle_mod.dist_knn3(pts), 1e-7)
    np.testing.assert_allclose(m._scaling.cpu().numpy(), np.repeat(np.log(np.sqrt(d2))[:, None], 3, 1), rtol=1e-5,
                               atol=1e-6)
    np.testing.assert_allclose(m._features_dc.cpu().numpy()[:, 0], (cols - 0.5) / 0.28209479177387814, rtol=1e-6)
    assert float(m._features_rest.abs().max()) == 0.0
    np.testing.assert_allclose(m.get_opacity.detach().cpu().numpy(), 0.1, rtol=1e-6)
    np.testing.assert_allclose(m.get_rotation.detach().cpu().numpy(), np.tile([1, 0, 0, 0], (3000, 1)))
