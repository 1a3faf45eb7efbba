"""Pin the CPU oracle (and the harness camera builder) against golden vectors
generated from the reference's own Python (tests/golden/make_golden.py):
eval_sh / RGB2SH (utils/sh_utils.py) and the camera matrices of
utils/graphics_utils.py + scene/cameras.py.  CPU only."""
import math
import os

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")


def _cam_from_golden(z, i):
    from gsr_tools.scene import make_camera
    W, H = (int(v) for v in z[f"cam{i}_size"])
    FoVx, FoVy = (float(v) for v in z[f"cam{i}_fov"])
    return make_camera(z[f"cam{i}_R"], z[f"cam{i}_T"], W, H, FoVx, FoVy)


def test_camera_matrices_match_reference():
    """gsr_tools.scene.make_camera == reference getWorld2View2/getProjectionMatrix
    with the scene/cameras.py:58-61 transposes (bitwise)."""
    z = np.load(os.path.join(GOLD, "camera_golden.npz"))
    for i in range(int(z["n_cams"])):
        cam = _cam_from_golden(z, i)
        np.testing.assert_array_equal(cam.world_view_transform.numpy(), z[f"cam{i}_world_view"])
        np.testing.assert_array_equal(cam.full_proj_transform.numpy(), z[f"cam{i}_full_proj"])
        np.testing.assert_array_equal(cam.camera_center.numpy(), z[f"cam{i}_center"])


def test_rgb2sh_matches_reference():
    from gsr_tools.scene import rgb2sh
    z = np.load(os.path.join(GOLD, "sh_golden.npz"))
    np.testing.assert_allclose(rgb2sh(torch.from_numpy(z["rgb2sh_in"])).numpy(), z["rgb2sh_out"], rtol=0, atol=0)


@pytest.mark.parametrize("deg", [0, 1, 2, 3])
def test_oracle_sh_colour_matches_reference_eval_sh(oracle_mod, deg):
    """Oracle rgb (forward.cu:20-71) == clamp_min(eval_sh(deg) + 0.5, 0) of the reference
    (utils/sh_utils.py:57-112 in float64) to fp32 rounding; the clamped mask matches
    exactly away from the clamp boundary."""
    from gsr_tools.scene import Scene, make_camera, focal2fov
    z = np.load(os.path.join(GOLD, "sh_golden.npz"))
    means = torch.from_numpy(z["means"])
    N = means.shape[0]
    g = torch.Generator().manual_seed(0)
    rots = torch.randn(N, 4, generator=g)
    rots = rots / rots.norm(dim=1, keepdim=True)
    scene = Scene(means, torch.from_numpy(z["shs"]), torch.full((N, 1), 0.5), torch.full((N, 3), 0.02), rots,
                  torch.full((N, 2), 0.5), deg)
    cam = make_camera(np.eye(3), np.array([0.0, 0.0, 4.0]), 256, 256, focal2fov(200.0, 256), focal2fov(200.0, 256))
    cam.camera_center = torch.from_numpy(z["campos"])  # SH view direction uses settings.campos only
    run = oracle_mod.run_scene(scene, cam)
    assert (run.radii > 0).all(), "golden scene must be fully visible"
    rgb = run.get("rgb").reshape(N, 3)
    ref = z[f"rgb_deg{deg}"]
    np.testing.assert_allclose(rgb, ref, rtol=0, atol=2e-6)
    clamped = run.get("clamped").reshape(N, 3).astype(bool)
    raw = z[f"eval_sh_deg{deg}"] + 0.5
    away = np.abs(raw) > 1e-5
    np.testing.assert_array_equal(clamped[away], (raw < 0)[away])


def test_oracle_mark_visible(oracle_mod):
    """markVisible: view-space z > 0.2 (auxiliary.h:154)."""
    from gsr_tools.scene import make_camera, focal2fov
    cam = make_camera(np.eye(3), np.array([0.0, 0.0, 1.0]), 64, 64, focal2fov(50.0, 64), focal2fov(50.0, 64))
    m = torch.tensor([[0, 0, 0.0], [0, 0, -0.79], [0, 0, -0.81], [5, 5, 3.0], [0, 0, -2.0]])
    vis = oracle_mod.mark_visible(m, cam.world_view_transform.numpy())
    assert vis.tolist() == [True, True, False, True, False]


def test_blend_exp_accuracy(oracle_mod):
    """gsr_expf (shared bit-for-bit by the oracle and the HIP kernels) is within 1 ulp of
    exp() on the blend's range [-5.6, 0] (powers at or above the opacity floor; exhaustive
    check: max 0.887 ulp, render.hip) and within 5 ulp on [-87, 88] (its one-FMA reduction
    loses |k| * 1.9e-9 at large |k|, where only rejected pairs land); it returns exp of the
    clamped argument outside.  The reference's CUDA expf is specified at 2 ulp."""
    rng = np.random.default_rng(0)
    blend = np.concatenate([-np.abs(rng.standard_normal(20000)) * 2.0, -rng.random(20000) * 5.6,
                            np.array([0.0, -0.0, -1e-30, -5.6])]).astype(np.float32)
    wide = np.concatenate([-rng.random(20000) * 87.0, rng.random(2000) * 88.0,
                           np.array([-87.0, 88.0])]).astype(np.float32)
    for xs, bound in ((blend, 1.0), (wide, 5.0)):
        got = np.array([oracle_mod.expf(x) for x in xs], dtype=np.float32)
        ref = np.exp(xs.astype(np.float64))
        ulp = np.spacing(ref.astype(np.float32)).astype(np.float64)
        normal = ref > 1.2e-38
        err = np.abs(got[normal].astype(np.float64) - ref[normal]) / ulp[normal]
        assert err.max() < bound, (bound, err.max())
    # outside the clamp: exp(-87) / exp(88) to within the same accuracy
    assert abs(oracle_mod.expf(-200.0) / math.exp(-87.0) - 1) < 1e-6
    assert abs(oracle_mod.expf(1000.0) / math.exp(88.0) - 1) < 1e-6


# ---- utils/general_utils.py (tests/golden/general_utils_golden.npz) ----------------

def _scene_of(means, scales, rots):
    from gsr_tools.scene import Scene
    N = means.shape[0]
    return Scene(means, torch.zeros(N, 1, 3), torch.full((N, 1), 0.5), scales, rots, torch.full((N, 2), 0.5), 0)


@pytest.mark.parametrize("tag,mod", [("1", 1.0), ("0p25", 0.25)])
def test_oracle_cov3d_matches_reference_covariance(oracle_mod, tag, mod):
    """Oracle cov3D (forward.cu:118-152: Sigma = (S R)^T (S R), S = diag(mod * s)) ==
    the reference's Python covariance, strip_symmetric(L L^T) with L =
    build_scaling_rotation(mod * s, q) (utils/general_utils.py:72-118 via
    scene/gaussian_model.py:28-32), for normalised quaternions: the two evaluate the
    same products in a different order, so they agree to a few fp32 ulps of the
    covariance's largest entry."""
    from gsr_tools.scene import make_camera, focal2fov
    z = np.load(os.path.join(GOLD, "general_utils_golden.npz"))
    scales = torch.from_numpy(z["scales"])
    rots = torch.from_numpy(z["rotations_normalized"])
    N = scales.shape[0]
    g = torch.Generator().manual_seed(3)
    means = (torch.rand(N, 3, generator=g) * 2 - 1) * 0.5  # in front of the camera: all preprocessed
    cam = make_camera(np.eye(3), np.array([0.0, 0.0, 4.0]), 256, 256, focal2fov(200.0, 256), focal2fov(200.0, 256))
    run = oracle_mod.run_scene(_scene_of(means, scales, rots), cam, scale_modifier=mod)
    cov = run.get("cov3D").reshape(N, 6).astype(np.float64)
    ref = z[f"cov3D_mod{tag}"].astype(np.float64)
    # float64 truth of the same formula, to tell whose rounding the difference is
    sd, qd = scales.double() * mod, rots.double()
    w, x, y, zq = qd.T
    R = torch.stack([1 - 2 * (y * y + zq * zq), 2 * (x * y - w * zq), 2 * (x * zq + w * y),
                     2 * (x * y + w * zq), 1 - 2 * (x * x + zq * zq), 2 * (y * zq - w * x),
                     2 * (x * zq - w * y), 2 * (y * zq + w * x), 1 - 2 * (x * x + y * y)], 1).view(N, 3, 3)
    Lm = R @ torch.diag_embed(sd)
    exact = (Lm @ Lm.transpose(1, 2))[:, [0, 0, 0, 1, 1, 2], [0, 1, 2, 1, 2, 2]].numpy()
    scale = np.abs(exact).max(1, keepdims=True)
    err = (np.abs(cov - ref) / scale).max()
    err_oracle, err_ref = (np.abs(cov - exact) / scale).max(), (np.abs(ref - exact) / scale).max()
    # measured: oracle vs reference 1.4e-6, oracle vs exact 4.0e-7, reference vs exact 1.3e-6
    # (the reference's L L^T rounds more than the CUDA (SR)^T(SR) order the oracle follows)
    assert err <= 2e-6, f"max |cov3D - reference| = {err:.2e} of the row's largest entry"
    assert err_oracle <= max(err_ref, 5e-7), f"oracle {err_oracle:.2e} vs reference {err_ref:.2e} from float64"


def test_train_oracle_build_rotation_matches_reference():
    """oracle/train_oracle.py _build_rotation (used by densify_and_split) == the
    reference's build_rotation (utils/general_utils.py:86-107), bitwise on the CPU."""
    from oracle.train_oracle import _build_rotation
    z = np.load(os.path.join(GOLD, "general_utils_golden.npz"))
    np.testing.assert_array_equal(_build_rotation(torch.from_numpy(z["rotations"])).numpy(), z["build_rotation"])


def test_lr_schedule_matches_reference():
    """gsr_train.get_expon_lr_func == the reference's get_expon_lr_func
    (utils/general_utils.py:37-70), bitwise (both float64 numpy)."""
    from gsr_train.gaussian_model import get_expon_lr_func
    z = np.load(os.path.join(GOLD, "general_utils_golden.npz"))
    for i, (a, b, d, m, n) in enumerate(z["lr_cases"]):
        f = get_expon_lr_func(lr_init=float(a), lr_final=float(b), lr_delay_steps=int(d), lr_delay_mult=float(m),
                              max_steps=int(n))
        got = np.array([float(f(int(s))) for s in z["lr_steps"]])
        np.testing.assert_array_equal(got, z[f"lr_case{i}"], err_msg=f"case {i}")
