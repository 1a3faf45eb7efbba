"""Reference camera conventions + synthetic Gaussian scenes.

Camera matrices mirror the reference exactly:
  * getWorld2View2 / getProjectionMatrix  (utils/graphics_utils.py:38-74)
  * world_view_transform = W2C^T, full_proj = world_view @ proj^T,
    camera_center = inverse(world_view)[3, :3]  (scene/cameras.py:58-61)
tests/golden/camera_*.npz pins this file against the reference's own functions.

Synthetic scenes follow SURVEY.md s8(d) (seeded CPU torch.Generator, fp32).
"""
import math
from dataclasses import dataclass

import numpy as np
import torch

SH_C0 = 0.28209479177387814  # utils/sh_utils.py:26


def rgb2sh(rgb):
    """utils/sh_utils.py:114-115"""
    return (rgb - 0.5) / SH_C0


def world2view2(R, t, translate=np.array([0.0, 0.0, 0.0]), scale=1.0):
    """utils/graphics_utils.py:38-49 (float64 numpy, float32 result)."""
    Rt = np.zeros((4, 4))
    Rt[:3, :3] = R.transpose()
    Rt[:3, 3] = t
    Rt[3, 3] = 1.0
    C2W = np.linalg.inv(Rt)
    cam_center = C2W[:3, 3]
    cam_center = (cam_center + translate) * scale
    C2W[:3, 3] = cam_center
    Rt = np.linalg.inv(C2W)
    return np.float32(Rt)


def projection_matrix(znear, zfar, fovX, fovY):
    """utils/graphics_utils.py:51-74 (torch float32)."""
    tanHalfFovY = math.tan((fovY / 2))
    tanHalfFovX = math.tan((fovX / 2))
    top = tanHalfFovY * znear
    bottom = -top
    right = tanHalfFovX * znear
    left = -right
    P = torch.zeros(4, 4)
    z_sign = 1.0
    P[0, 0] = 2.0 * znear / (right - left)
    P[1, 1] = 2.0 * znear / (top - bottom)
    P[0, 2] = (right + left) / (right - left)
    P[1, 2] = (top + bottom) / (top - bottom)
    P[3, 2] = z_sign
    P[2, 2] = z_sign * zfar / (zfar - znear)
    P[2, 3] = -(zfar * znear) / (zfar - znear)
    return P


def focal2fov(focal, pixels):
    """utils/graphics_utils.py:79-80"""
    return 2 * math.atan(pixels / (2 * focal))


@dataclass
class Camera:
    width: int
    height: int
    FoVx: float
    FoVy: float
    world_view_transform: torch.Tensor  # [4,4] f32 (W2C^T)
    full_proj_transform: torch.Tensor   # [4,4] f32
    camera_center: torch.Tensor         # [3] f32

    @property
    def tanfovx(self):
        return math.tan(self.FoVx * 0.5)

    @property
    def tanfovy(self):
        return math.tan(self.FoVy * 0.5)

    def to(self, device):
        return Camera(self.width, self.height, self.FoVx, self.FoVy,
                      self.world_view_transform.to(device), self.full_proj_transform.to(device),
                      self.camera_center.to(device))


def make_camera(R, T, width, height, FoVx, FoVy, znear=0.01, zfar=100.0):
    """scene/cameras.py:52-61 on the CPU."""
    wv = torch.tensor(world2view2(np.asarray(R, dtype=np.float64), np.asarray(T, dtype=np.float64))).transpose(0, 1)
    pr = projection_matrix(znear=znear, zfar=zfar, fovX=FoVx, fovY=FoVy).transpose(0, 1)
    full = (wv.unsqueeze(0).bmm(pr.unsqueeze(0))).squeeze(0)
    center = wv.inverse()[3, :3]
    return Camera(width, height, FoVx, FoVy, wv.contiguous(), full.contiguous(), center.contiguous())


def orbit_camera(view_index, width, height, focal, radius=4.0, n_views=8):
    """Camera `view_index` of a horizontal orbit around the origin at `radius`
    (view 0 is R = I, T = (0, 0, radius): SURVEY.md s8(d))."""
    ang = 2.0 * math.pi * view_index / max(1, n_views)
    c, s = math.cos(ang), math.sin(ang)
    # world->camera rotation about y; R passed to getWorld2View2 is its transpose (C2W rotation).
    Rw2c = np.array([[c, 0.0, -s], [0.0, 1.0, 0.0], [s, 0.0, c]])
    return make_camera(Rw2c.T, np.array([0.0, 0.0, radius]), width, height,
                       focal2fov(focal, width), focal2fov(focal, height))


@dataclass
class Scene:
    means3D: torch.Tensor
    shs: torch.Tensor
    opacities: torch.Tensor
    scales: torch.Tensor
    rotations: torch.Tensor
    segments: torch.Tensor
    sh_degree: int

    @property
    def P(self):
        return self.means3D.shape[0]

    def to(self, device):
        return Scene(*(getattr(self, f).to(device) for f in
                       ("means3D", "shs", "opacities", "scales", "rotations", "segments")), self.sh_degree)


def synthetic_scene(P, sh_degree=3, extent=1.5, log_scale=math.log(0.01), log_scale_std=0.5,
                    seed=0, n_classes=2):
    """SURVEY.md s8(d) generator: means ~ U[-e,e]^3, scales = exp(N(log_scale, std)),
    rotations = normalize(N(0,1)^4), opacity = sigmoid(N(0,1)), segments = sigmoid(N(0,1)),
    SH DC = RGB2SH(U[0,1]), rest N(0, 0.05)."""
    g = torch.Generator().manual_seed(seed)
    M = (sh_degree + 1) ** 2
    # exp / sigmoid / norm in float64, rounded once: torch's float32 CPU kernels differ in the
    # last bit between CPUs (the GPU box's EPYC and this container's Xeon gave different
    # scales and opacities), which made the "same" scene differ between machines
    f64 = lambda t: t.to(torch.float64)
    means = (torch.rand(P, 3, generator=g) * 2 - 1) * extent
    scales = torch.exp(f64(torch.randn(P, 3, generator=g)) * log_scale_std + log_scale).float()
    rots = f64(torch.randn(P, 4, generator=g))
    rots = (rots / rots.norm(dim=1, keepdim=True)).float()
    opac = torch.sigmoid(f64(torch.randn(P, 1, generator=g))).float()
    segs = torch.sigmoid(f64(torch.randn(P, n_classes, generator=g))).float()
    shs = torch.zeros(P, M, 3)
    shs[:, 0, :] = rgb2sh(torch.rand(P, 3, generator=g))
    if M > 1:
        shs[:, 1:, :] = torch.randn(P, M - 1, 3, generator=g) * 0.05
    return Scene(means.contiguous(), shs.contiguous(), opac.contiguous(), scales.contiguous(),
                 rots.contiguous(), segs.contiguous(), sh_degree)


# Named configurations of BASELINE.json / SURVEY.md s8(d).
CONFIGS = {
    # C1: 10k, SH0, 256^2, FoV 60 deg, scale ln 0.02
    "c1": dict(P=10_000, sh_degree=0, width=256, height=256, fov_deg=60.0, log_scale=math.log(0.02), extent=1.5),
    # C2: lego-like 300k, SH3, 800^2, focal 1111, U[-1.3,1.3]^3
    "c2": dict(P=300_000, sh_degree=3, width=800, height=800, focal=1111.0, extent=1.3),
    # Metric: 1M, SH3, 1920x1080, focal 1200
    "mt": dict(P=1_000_000, sh_degree=3, width=1920, height=1080, focal=1200.0, extent=1.5),
    # C3: garden-like 3M, SH3, 1080p
    "c3": dict(P=3_000_000, sh_degree=3, width=1920, height=1080, focal=1200.0, extent=1.5),
    # C5: 6M = two 3M scenes merged (visualizer.py:196-226), SH3, 1080p
    "c5": dict(P=3_000_000, sh_degree=3, width=1920, height=1080, focal=1200.0, extent=1.5, merge=2),
}


def config_scene_and_camera(name, view_index=0, n_views=8, P=None, seed=0):
    c = dict(CONFIGS[name])
    if P is not None:
        c["P"] = P
    kw = {}
    if "log_scale" in c:
        kw["log_scale"] = c["log_scale"]
    scene = synthetic_scene(c["P"], sh_degree=c["sh_degree"], extent=c["extent"], seed=seed, **kw)
    for m in range(1, c.get("merge", 1)):  # concatenate independently seeded scenes
        other = synthetic_scene(c["P"], sh_degree=c["sh_degree"], extent=c["extent"], seed=seed + m, **kw)
        scene = Scene(*(torch.cat([getattr(scene, f), getattr(other, f)], 0).contiguous()
                        for f in ("means3D", "shs", "opacities", "scales", "rotations", "segments")),
                      scene.sh_degree)
    W, H = c["width"], c["height"]
    if "focal" in c:
        focal = c["focal"]
    else:
        focal = W / (2 * math.tan(math.radians(c["fov_deg"]) / 2))
    cam = orbit_camera(view_index, W, H, focal, n_views=n_views)
    return scene, cam
