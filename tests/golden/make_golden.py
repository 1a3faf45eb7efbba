"""Generate golden vectors from the reference's own importable Python.

Runs ONLY in the build container (needs /root/reference; never on the GPU box):
    python -B tests/golden/make_golden.py
Writes small .npz fixtures next to this script.  The reference code is imported,
never copied:
  * utils/sh_utils.py  eval_sh (:57-112), RGB2SH (:114-115)
  * utils/graphics_utils.py  getWorld2View2 (:38-49), getProjectionMatrix (:51-74),
    focal2fov (:79-80), with the scene/cameras.py:58-61 transposes.
  * utils/general_utils.py  build_rotation (:86-107), build_scaling_rotation (:109-118),
    strip_symmetric (:72-84), get_expon_lr_func (:37-70).  The module allocates with a
    hard-coded device="cuda"; it runs here on the CPU through a shim that drops that
    keyword from torch.zeros for the duration of the calls (the module is imported
    unchanged, nothing of it is copied).
"""
import math
import os
import sys

sys.dont_write_bytecode = True  # never write __pycache__ into /root/reference
REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))

import numpy as np
import torch

sys.path.insert(0, REF)
from utils.sh_utils import eval_sh, RGB2SH  # noqa: E402  (reference code)
from utils.graphics_utils import getWorld2View2, getProjectionMatrix, focal2fov  # noqa: E402
import utils.general_utils as GU  # noqa: E402  (reference code)
sys.path.remove(REF)


class _CpuTorch:
    """torch, except that torch.zeros ignores device= (general_utils hard-codes "cuda")."""

    def __getattr__(self, name):
        return getattr(torch, name)

    @staticmethod
    def zeros(*args, **kw):
        kw.pop("device", None)
        return torch.zeros(*args, **kw)


class _cpu_general_utils:
    def __enter__(self):
        self.saved = GU.torch
        GU.torch = _CpuTorch()

    def __exit__(self, *exc):
        GU.torch = self.saved


def reference_covariance(scaling, scaling_modifier, rotation):
    """scene/gaussian_model.py:28-32 (build_covariance_from_scaling_rotation) over the
    reference's own build_scaling_rotation / strip_symmetric."""
    with _cpu_general_utils():
        L = GU.build_scaling_rotation(scaling_modifier * scaling, rotation)
        return GU.strip_symmetric(L @ L.transpose(1, 2))


def reference_colors(means, shs, campos, degree):
    """gaussian_renderer/__init__.py:341-357 (convert_SHs_python): float32 like the
    reference, shs in the rasterizer layout [P, M, 3]."""
    M = shs.shape[1]
    shs_view = shs.transpose(1, 2).view(-1, 3, M)
    dir_pp = means - campos.repeat(shs.shape[0], 1)
    dir_pp_normalized = dir_pp / dir_pp.norm(dim=1, keepdim=True)
    sh2rgb = eval_sh(degree, shs_view, dir_pp_normalized)
    return torch.clamp_min(sh2rgb + 0.5, 0.0)


def sh_vectors():
    """SH -> RGB in the rasterizer's convention: rgb = max(eval_sh(deg, sh, dir) + 0.5, 0)
    with dir = (mean - campos) / |mean - campos| (forward.cu:25-27,63-70).  The
    directions are formed in float32 exactly as the kernel forms them; eval_sh runs
    in float64 on the reference's own code."""
    g = torch.Generator().manual_seed(11)
    N = 257
    means = (torch.rand(N, 3, generator=g) * 2 - 1) * 1.5
    campos = torch.tensor([0.3, -0.2, -4.0])
    shs = torch.randn(N, 16, 3, generator=g) * 0.3  # [P, M, 3] rasterizer layout
    shs[:, 0, :] = RGB2SH(torch.rand(N, 3, generator=g))
    d32 = (means - campos).numpy().astype(np.float32)
    n32 = np.sqrt((d32 * d32).sum(1, dtype=np.float32)).astype(np.float32)  # x*x+y*y+z*z, sqrt
    dirs = (d32 / n32[:, None]).astype(np.float32)
    out = {"means": means.numpy(), "campos": campos.numpy(), "shs": shs.numpy(), "dirs": dirs}
    sh_view = shs.double().transpose(1, 2)  # [..., C, coeffs] as eval_sh expects (gaussian_renderer:353)
    for deg in range(4):
        val = eval_sh(deg, sh_view, torch.from_numpy(dirs).double())
        out[f"eval_sh_deg{deg}"] = val.numpy()
        out[f"rgb_deg{deg}"] = torch.clamp_min(val + 0.5, 0.0).numpy()
    rgb = torch.rand(16, 3, generator=g)
    out["rgb2sh_in"] = rgb.numpy()
    out["rgb2sh_out"] = RGB2SH(rgb).numpy()
    np.savez_compressed(os.path.join(HERE, "sh_golden.npz"), **out)


def camera_vectors():
    """world_view_transform / full_proj_transform / camera_center as scene/cameras.py:58-61
    builds them from the reference's getWorld2View2 + getProjectionMatrix."""
    out = {}
    cams = []
    for i, (W, H, focal) in enumerate([(1920, 1080, 1200.0), (800, 800, 1111.0), (256, 256, 221.7025033688164),
                                       (333, 250, 300.0)]):
        ang = 2.0 * math.pi * i / 8
        c, s = math.cos(ang), math.sin(ang)
        Rw2c = np.array([[c, 0.0, -s], [0.0, 1.0, 0.0], [s, 0.0, c]])
        R = Rw2c.T
        T = np.array([0.1 * i, -0.05 * i, 4.0])
        FoVx, FoVy = focal2fov(focal, W), focal2fov(focal, H)
        wv = torch.tensor(getWorld2View2(R, T, np.array([0.0, 0.0, 0.0]), 1.0)).transpose(0, 1)
        pr = getProjectionMatrix(znear=0.01, zfar=100.0, fovX=FoVx, fovY=FoVy).transpose(0, 1)
        full = (wv.unsqueeze(0).bmm(pr.unsqueeze(0))).squeeze(0)
        center = wv.inverse()[3, :3]
        out[f"cam{i}_R"] = R
        out[f"cam{i}_T"] = T
        out[f"cam{i}_size"] = np.array([W, H])
        out[f"cam{i}_fov"] = np.array([FoVx, FoVy])
        out[f"cam{i}_world_view"] = wv.numpy()
        out[f"cam{i}_full_proj"] = full.numpy()
        out[f"cam{i}_center"] = center.numpy()
        cams.append(i)
    out["n_cams"] = np.array(len(cams))
    np.savez_compressed(os.path.join(HERE, "camera_golden.npz"), **out)


def general_utils_vectors():
    """build_rotation, the covariance of build_scaling_rotation + strip_symmetric and
    get_expon_lr_func, evaluated by the reference's own functions (float32 on the CPU)."""
    g = torch.Generator().manual_seed(13)
    N = 512
    rots = torch.randn(N, 4, generator=g)
    rots_n = rots / rots.norm(dim=1, keepdim=True)
    scales = torch.exp(torch.randn(N, 3, generator=g) * 0.8 + math.log(0.02))
    out = {"rotations": rots.numpy(), "rotations_normalized": rots_n.numpy(), "scales": scales.numpy()}
    with _cpu_general_utils():
        out["build_rotation"] = GU.build_rotation(rots).numpy()
    for tag, mod in (("1", 1.0), ("0p25", 0.25)):
        out[f"cov3D_mod{tag}"] = reference_covariance(scales, mod, rots_n).numpy()
    # learning-rate schedules (train.py / arguments defaults: position lr 1.6e-4 -> 1.6e-6 over
    # 30k steps scaled by the scene extent, delay multiplier 0.01) plus a delayed warm-up case
    steps = np.array([-1, 0, 1, 2, 10, 100, 999, 1000, 1001, 5000, 7000, 15000, 29999, 30000, 30001, 100000])
    cases = [(0.00016 * 4.2, 0.0000016 * 4.2, 0, 0.01, 30000), (0.0025, 0.0025, 0, 1.0, 30000),
             (0.01, 0.0001, 1000, 0.01, 30000), (0.0, 0.0, 0, 1.0, 30000), (0.001, 0.00001, 500, 0.1, 20000)]
    out["lr_steps"] = steps
    out["lr_cases"] = np.array(cases, dtype=np.float64)
    for i, (a, b, d, m, n) in enumerate(cases):
        f = GU.get_expon_lr_func(lr_init=a, lr_final=b, lr_delay_steps=int(d), lr_delay_mult=m, max_steps=int(n))
        out[f"lr_case{i}"] = np.array([float(f(int(st))) for st in steps], dtype=np.float64)
    np.savez_compressed(os.path.join(HERE, "general_utils_golden.npz"), **out)


def render_path_vectors():
    """The reference's Python argument paths of render() (gaussian_renderer/__init__.py:
    241-263 and 326-357): cov3D_precomp from get_covariance (compute_cov3D_python) and
    colors_precomp from eval_sh (convert_SHs_python), for a seeded scene and camera; the
    GPU test feeds them to the HIP path and compares with the oracle's internal
    scales/rotations and SH evaluation."""
    g = torch.Generator().manual_seed(17)
    P = 3000
    means = ((torch.rand(P, 3, generator=g) * 2 - 1) * 1.2).float()
    scales = torch.exp(torch.randn(P, 3, generator=g) * 0.5 + math.log(0.03))
    rots = torch.randn(P, 4, generator=g)
    rots = rots / rots.norm(dim=1, keepdim=True)
    opac = torch.sigmoid(torch.randn(P, 1, generator=g))
    segs = torch.sigmoid(torch.randn(P, 2, generator=g))
    shs = torch.randn(P, 16, 3, generator=g) * 0.1
    shs[:, 0, :] = RGB2SH(torch.rand(P, 3, generator=g))
    W, H, focal = 320, 240, 280.0
    ang = 2.0 * math.pi * 3 / 8
    c, s = math.cos(ang), math.sin(ang)
    R = np.array([[c, 0.0, -s], [0.0, 1.0, 0.0], [s, 0.0, c]]).T
    T = np.array([0.05, -0.1, 4.0])
    FoVx, FoVy = focal2fov(focal, W), focal2fov(focal, H)
    wv = torch.tensor(getWorld2View2(R, T, np.array([0.0, 0.0, 0.0]), 1.0)).transpose(0, 1)
    pr = getProjectionMatrix(znear=0.01, zfar=100.0, fovX=FoVx, fovY=FoVy).transpose(0, 1)
    full = (wv.unsqueeze(0).bmm(pr.unsqueeze(0))).squeeze(0)
    center = wv.inverse()[3, :3]
    out = {"means3D": means.numpy(), "scales": scales.numpy(), "rotations": rots.numpy(),
           "opacities": opac.numpy(), "segments": segs.numpy(), "shs": shs.numpy(),
           "size": np.array([W, H]), "fov": np.array([FoVx, FoVy]), "world_view": wv.numpy(),
           "full_proj": full.numpy(), "center": center.numpy()}
    for mod, tag in ((1.0, "1"), (0.7, "0p7")):
        out[f"cov3D_precomp_mod{tag}"] = reference_covariance(scales, mod, rots).numpy()
    for deg in (0, 1, 3):
        out[f"colors_precomp_deg{deg}"] = reference_colors(means, shs, center, deg).numpy()
    np.savez_compressed(os.path.join(HERE, "render_paths_golden.npz"), **out)


if __name__ == "__main__":
    sh_vectors()
    camera_vectors()
    general_utils_vectors()
    render_path_vectors()
    print("wrote", sorted(f for f in os.listdir(HERE) if f.endswith(".npz")))
