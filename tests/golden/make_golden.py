"""Generate golden vectors from the reference's own importable Python.

Runs ONLY in the build container (needs /root/reference; never on the GPU box):
    python -B tests/golden/make_golden.py
Writes small .npz fixtures next to this script.  The reference code is imported,
never copied:
  * utils/sh_utils.py  eval_sh (:57-112), RGB2SH (:114-115)
  * utils/graphics_utils.py  getWorld2View2 (:38-49), getProjectionMatrix (:51-74),
    focal2fov (:79-80), with the scene/cameras.py:58-61 transposes.
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
sys.path.remove(REF)


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


if __name__ == "__main__":
    sh_vectors()
    camera_vectors()
    print("wrote", sorted(f for f in os.listdir(HERE) if f.endswith(".npz")))
