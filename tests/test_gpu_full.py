"""Full-size parity at the BASELINE metric configuration (1M Gaussians, SH3, 1920x1080):
bit-exact integer outputs and image/gradient tolerances as in test_gpu_parity.py,
plus size-independent structural properties of the binning."""
import numpy as np
import pytest

import harness as Hn
from gsr_tools.scene import config_scene_and_camera
from test_gpu_parity import assert_integer_parity, assert_image_parity, assert_grad_parity

pytestmark = [pytest.mark.gpu, pytest.mark.slow]


@pytest.fixture(scope="module")
def mt_runs(oracle_mod):
    scene, cam = config_scene_and_camera("mt")
    grads = Hn.upstream_grads(cam.height, cam.width)
    g = Hn.run_gsr(scene, cam, grads=grads)
    r = Hn.run_oracle(oracle_mod, scene, cam, grads=grads)
    return scene, cam, g, r


def test_metric_config_integer_parity(gpu_available, mt_runs):
    scene, cam, g, r = mt_runs
    assert g["num_rendered"] > 5_000_000
    assert_integer_parity(g, r)


def test_metric_config_image_parity(gpu_available, mt_runs):
    assert_image_parity(mt_runs[2], mt_runs[3])


def test_metric_config_grad_parity(gpu_available, mt_runs):
    assert_grad_parity(mt_runs[2]["grads"], mt_runs[3]["grads"])


def test_binning_properties(gpu_available, mt_runs):
    """ranges partition [0, I) in tile order; inside a tile the list is sorted by
    (depth bits, gaussian id); every instance's tile lies in its Gaussian's rectangle."""
    scene, cam, g, r = mt_runs
    I = g["num_rendered"]
    ranges = g["ranges"].reshape(-1, 2).astype(np.int64)
    nonempty = ranges[:, 1] > ranges[:, 0]
    starts, ends = ranges[nonempty, 0], ranges[nonempty, 1]
    assert starts[0] == 0 and ends[-1] == I
    np.testing.assert_array_equal(starts[1:], ends[:-1])
    assert int(g["tiles_touched"].astype(np.int64).sum()) == I
    pl = g["point_list"].astype(np.int64)
    rec = g["rec"].reshape(-1, 16)
    depth_bits = rec[:, 6].view(np.uint32).astype(np.uint64)
    key = (depth_bits[pl] << np.uint64(32)) | pl.astype(np.uint64)
    tile_of = np.repeat(np.nonzero(nonempty)[0], ends - starts)
    same = tile_of[1:] == tile_of[:-1]
    assert np.all(key[1:][same] > key[:-1][same])
