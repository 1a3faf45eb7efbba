"""Full-size parity at every single-GPU BASELINE configuration -- the metric config
(1M Gaussians, SH3, 1920x1080), C2 (300k, 800x800), C3 (3M, 1080p; I ~ 24M) and C5 (two
3M scenes merged, 6M Gaussians; I ~ 48M, P > 4M takes the depth sort's table passes):
bit-exact integer outputs (num_rendered, radii, tiles_touched, point_list, ranges,
n_contrib) and the image / scale-free gradient tolerances of test_gpu_parity.py, plus
size-independent structural properties of the binning (the 45-bit key order of
rasterizer_impl.cu:304-312 at tens of millions of instances).  C4 (8 views on 8 GPUs)
is the multi-GPU sharding of C3 and is exercised by the driver's scaling run."""
import numpy as np
import pytest

import harness as Hn
from gsr_tools.scene import config_scene_and_camera
from test_gpu_parity import assert_integer_parity, assert_image_parity, assert_grad_parity

pytestmark = [pytest.mark.gpu, pytest.mark.slow]


# config -> minimum num_rendered (guards against a scene that silently shrank)
MIN_INSTANCES = {"mt": 5_000_000, "c2": 1_000_000, "c3": 15_000_000, "c5": 30_000_000}


@pytest.fixture(scope="module", params=["mt", "c2", "c3", "c5"])
def mt_runs(request, oracle_mod):
    scene, cam = config_scene_and_camera(request.param)
    grads = Hn.upstream_grads(cam.height, cam.width)
    g = Hn.run_gsr(scene, cam, grads=grads)
    r = Hn.run_oracle(oracle_mod, scene, cam, grads=grads)
    r["noise"] = Hn.reference_noise(oracle_mod, r.pop("_run"), grads, r["grads"])
    yield request.param, scene, cam, g, r


def test_full_config_integer_parity(gpu_available, mt_runs):
    name, scene, cam, g, r = mt_runs
    assert g["num_rendered"] > MIN_INSTANCES[name]
    assert_integer_parity(g, r)


def test_full_config_image_parity(gpu_available, mt_runs):
    assert_image_parity(mt_runs[3], mt_runs[4])


def test_full_config_grad_parity(gpu_available, mt_runs):
    """Scale-free 1e-5, or 4x the reference's own fp32-order deviation where that is larger
    (assert_grad_parity; printed per tensor)."""
    r = mt_runs[4]
    print(f"\n{mt_runs[0]}: reference fp32-order deviation " + ", ".join(f"{k} {v:.1e}" for k, v in r["noise"].items()))
    assert_grad_parity(mt_runs[3]["grads"], r["grads"], r["noise"])


def test_binning_properties(gpu_available, mt_runs):
    """ranges partition [0, I) in tile order; inside a tile the list is sorted by
    (depth bits, gaussian id); every instance's tile lies in its Gaussian's rectangle."""
    name, scene, cam, g, r = mt_runs
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
    # getRect (auxiliary.h:46-56): float arithmetic, (int) truncation, clamp to [0, grid]
    gx, gy = (cam.width + 15) // 16, (cam.height + 15) // 16
    rad = g["radii"].astype(np.float32)
    px, py = rec[:, 0].astype(np.float32), rec[:, 1].astype(np.float32)
    f16 = np.float32(16)
    rect = lambda v, n: np.clip(np.trunc(v).astype(np.int64), 0, n)
    x0, x1 = rect((px - rad) / f16, gx), rect((px + rad + np.float32(15)) / f16, gx)
    y0, y1 = rect((py - rad) / f16, gy), rect((py + rad + np.float32(15)) / f16, gy)
    tx, ty = tile_of % gx, tile_of // gx
    assert np.all((tx >= x0[pl]) & (tx < x1[pl]) & (ty >= y0[pl]) & (ty < y1[pl]))
    np.testing.assert_array_equal((x1 - x0) * (y1 - y0) * (g["radii"] > 0), g["tiles_touched"].astype(np.int64))
