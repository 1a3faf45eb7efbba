"""Pin the oracle's forward and hand-derived backward (restating backward.cu) against
a float64 PyTorch-autograd restatement of the same mathematics (CPU only).

The restatement re-derives every differentiable quantity from the inputs in fp64
(projection, EWA covariance, SH colour, alpha compositing) and takes only the
non-differentiable structure (per-tile sorted lists) from the oracle.  Scenes are
kept inside the regime where the reference's gradient is the true gradient:
no tx/tz frustum clamp (backward.cu:175-176), opacity*G < 0.99 (alpha clamp,
backward.cu:548), bg arbitrary.
"""
import math

import numpy as np
import pytest
import torch

from gsr_tools.scene import Scene, make_camera, focal2fov

C0 = 0.28209479177387814
C1 = 0.4886025119029199
C2 = [1.0925484305920792, -1.0925484305920792, 0.31539156525252005, -1.0925484305920792, 0.5462742152960396]
C3 = [-0.5900435899266435, 2.890611442640554, -0.4570457994644658, 0.3731763325901154, -0.4570457994644658,
      1.445305721320277, -0.5900435899266435]


def sh_basis(deg, d):
    x, y, z = d[:, 0], d[:, 1], d[:, 2]
    b = [torch.full_like(x, C0)]
    if deg > 0:
        b += [-C1 * y, C1 * z, -C1 * x]
    if deg > 1:
        xx, yy, zz, xy, yz, xz = x * x, y * y, z * z, x * y, y * z, x * z
        b += [C2[0] * xy, C2[1] * yz, C2[2] * (2 * zz - xx - yy), C2[3] * xz, C2[4] * (xx - yy)]
    if deg > 2:
        b += [C3[0] * y * (3 * xx - yy), C3[1] * xy * z, C3[2] * y * (4 * zz - xx - yy),
              C3[3] * z * (2 * zz - 3 * xx - 3 * yy), C3[4] * x * (4 * zz - xx - yy), C3[5] * z * (xx - yy),
              C3[6] * x * (xx - 3 * yy)]
    return torch.stack(b, 1)  # [P, (deg+1)^2]


def quat_to_rot(q):
    r, x, y, z = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    return torch.stack([
        torch.stack([1 - 2 * (y * y + z * z), 2 * (x * y - r * z), 2 * (x * z + r * y)], 1),
        torch.stack([2 * (x * y + r * z), 1 - 2 * (x * x + z * z), 2 * (y * z - r * x)], 1),
        torch.stack([2 * (x * z - r * y), 2 * (y * z + r * x), 1 - 2 * (x * x + y * y)], 1)], 1)


def restated_render(run, cam, inp, deg, bg, scale_modifier):
    """fp64 differentiable restatement; structure (point_list, ranges, radii) from the oracle run."""
    W, H = cam.width, cam.height
    view = torch.tensor(cam.world_view_transform.numpy(), dtype=torch.float64)  # W2C^T
    proj = torch.tensor(cam.full_proj_transform.numpy(), dtype=torch.float64)
    campos = torch.tensor(cam.camera_center.numpy(), dtype=torch.float64)
    m = inp["means3D"]
    P = m.shape[0]
    hom = torch.cat([m, torch.ones(P, 1, dtype=m.dtype)], 1)
    p_view = hom @ view  # row-vector convention of transformPoint4x3
    p_hom = hom @ proj
    p_w = 1.0 / (p_hom[:, 3] + 1e-7)
    ndc = p_hom[:, :2] * p_w[:, None] + inp["means2D"]  # means2D: the reference's dummy screen-space input
    pix = ((ndc + 1.0) * torch.tensor([W, H], dtype=m.dtype) - 1.0) * 0.5
    depth = p_view[:, 2]
    if "cov3D_precomp" in inp:
        c = inp["cov3D_precomp"]
        Sigma = torch.stack([torch.stack([c[:, 0], c[:, 1], c[:, 2]], 1), torch.stack([c[:, 1], c[:, 3], c[:, 4]], 1),
                             torch.stack([c[:, 2], c[:, 4], c[:, 5]], 1)], 1)
    else:
        Rq = quat_to_rot(inp["rotations"])
        Mm = torch.diag_embed(scale_modifier * inp["scales"]) @ Rq.transpose(1, 2)
        Sigma = Mm.transpose(1, 2) @ Mm
    fx, fy = W / (2 * cam.tanfovx), H / (2 * cam.tanfovy)
    tx, ty, tz = p_view[:, 0], p_view[:, 1], p_view[:, 2]
    Rw = view[:3, :3].T
    J = torch.zeros(P, 3, 3, dtype=m.dtype)
    J[:, 0, 0] = fx / tz
    J[:, 0, 2] = -(fx * tx) / (tz * tz)
    J[:, 1, 1] = fy / tz
    J[:, 1, 2] = -(fy * ty) / (tz * tz)
    Tm = J @ Rw
    cov = Tm @ Sigma @ Tm.transpose(1, 2)
    a, b, cc = cov[:, 0, 0] + 0.3, cov[:, 0, 1], cov[:, 1, 1] + 0.3
    det = a * cc - b * b
    conic = torch.stack([cc / det, -b / det, a / det], 1)
    if "colors_precomp" in inp:
        rgb = inp["colors_precomp"]
    else:
        d = m - campos
        d = d / d.norm(dim=1, keepdim=True)
        basis = sh_basis(deg, d)
        rgb = torch.clamp_min((basis[:, :, None] * inp["shs"][:, : basis.shape[1], :]).sum(1) + 0.5, 0.0)
    opac = inp["opacities"][:, 0]
    segs = inp["segments"]
    point_list = run.get("point_list").astype(np.int64)
    ranges = run.get("ranges").reshape(-1, 2)
    gx = (W + 15) // 16
    color = torch.zeros(3, H, W, dtype=m.dtype)
    out_d = torch.zeros(H, W, dtype=m.dtype)
    out_a = torch.zeros(H, W, dtype=m.dtype)
    out_s = torch.zeros(2, H, W, dtype=m.dtype)
    bg = torch.tensor(bg, dtype=m.dtype)
    color_list, depth_list, alpha_list, seg_list, idx_list = [], [], [], [], []
    for t in range(ranges.shape[0]):
        x0, y0 = (t % gx) * 16, (t // gx) * 16
        ys, xs = torch.meshgrid(torch.arange(y0, min(y0 + 16, H)), torch.arange(x0, min(x0 + 16, W)),
                                indexing="ij")
        ys, xs = ys.reshape(-1), xs.reshape(-1)
        pxf, pyf = xs.to(m.dtype), ys.to(m.dtype)
        n = len(xs)
        Tr = torch.ones(n, dtype=m.dtype)
        C = torch.zeros(n, 3, dtype=m.dtype)
        S = torch.zeros(n, 2, dtype=m.dtype)
        Dd = torch.zeros(n, dtype=m.dtype)
        Wt = torch.zeros(n, dtype=m.dtype)
        done = torch.zeros(n, dtype=torch.bool)
        for k in range(int(ranges[t, 0]), int(ranges[t, 1])):
            g = int(point_list[k])
            dx, dy = pix[g, 0] - pxf, pix[g, 1] - pyf
            power = -0.5 * (conic[g, 0] * dx * dx + conic[g, 2] * dy * dy) - conic[g, 1] * dx * dy
            alpha = opac[g] * torch.exp(power)
            use = (~done) & (power <= 0) & (alpha >= 1.0 / 255.0)
            test_T = Tr * (1 - alpha)
            term = use & (test_T < 1e-4)
            done = done | term
            use = use & ~term
            w = torch.where(use, alpha * Tr, torch.zeros_like(alpha))
            C = C + w[:, None] * rgb[g][None, :]
            S = S + w[:, None] * segs[g][None, :]
            Dd = Dd + w * depth[g]
            Wt = Wt + w
            Tr = torch.where(use, test_T, Tr)
        idx_list.append(ys * W + xs)
        color_list.append(C + Tr[:, None] * bg[None, :])
        depth_list.append(Dd)
        alpha_list.append(Wt)
        seg_list.append(S)
    idx = torch.cat(idx_list)
    color = color.reshape(3, -1).index_put((torch.arange(3)[:, None], idx[None, :]), torch.cat(color_list).T)
    out_d = out_d.reshape(-1).index_put((idx,), torch.cat(depth_list))
    out_a = out_a.reshape(-1).index_put((idx,), torch.cat(alpha_list))
    out_s = out_s.reshape(2, -1).index_put((torch.arange(2)[:, None], idx[None, :]), torch.cat(seg_list).T)
    return color.reshape(3, H, W), out_d.reshape(1, H, W), out_a.reshape(1, H, W), out_s.reshape(2, H, W)


def small_scene(P, deg, seed):
    g = torch.Generator().manual_seed(seed)
    M = 16
    means = torch.rand(P, 3, generator=g) * torch.tensor([1.6, 1.2, 1.0]) - torch.tensor([0.8, 0.6, 0.5])
    scales = torch.exp(torch.randn(P, 3, generator=g) * 0.3 + math.log(0.06))
    rots = torch.randn(P, 4, generator=g)
    rots = rots / rots.norm(dim=1, keepdim=True)
    opac = 0.1 + 0.8 * torch.rand(P, 1, generator=g)
    segs = torch.rand(P, 2, generator=g)
    shs = torch.randn(P, M, 3, generator=g) * 0.2
    shs[:, 0] = (torch.rand(P, 3, generator=g) - 0.5) / C0
    return Scene(means, shs, opac, scales, rots, segs, deg)


CASES = [
    dict(name="sh3", deg=3, bg=(0.0, 0.0, 0.0), mod=1.0),
    dict(name="sh1_bg", deg=1, bg=(0.3, 0.1, 0.7), mod=0.8),
    dict(name="colors", deg=0, bg=(0.0, 0.2, 0.0), mod=1.0, colors=True),
    dict(name="cov3d", deg=2, bg=(0.0, 0.0, 0.0), mod=1.0, cov=True),
]


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_oracle_backward_is_the_true_gradient(oracle_mod, case):
    scene = small_scene(40, case["deg"], seed=7)
    W, H = 72, 40
    cam = make_camera(np.eye(3), np.array([0.0, 0.0, 3.0]), W, H, focal2fov(60.0, W), focal2fov(60.0, H))
    gcol = torch.Generator().manual_seed(3)
    colors = torch.rand(scene.P, 3, generator=gcol) if case.get("colors") else None
    cov = None
    if case.get("cov"):
        Rq = quat_to_rot(scene.rotations.double())
        Mm = torch.diag_embed(scene.scales.double()) @ Rq.transpose(1, 2)
        Sg = (Mm.transpose(1, 2) @ Mm).float()
        cov = torch.stack([Sg[:, 0, 0], Sg[:, 0, 1], Sg[:, 0, 2], Sg[:, 1, 1], Sg[:, 1, 2], Sg[:, 2, 2]], 1)
    run = oracle_mod.run_scene(scene, cam, bg=case["bg"], scale_modifier=case["mod"], colors_precomp=colors,
                               cov3D_precomp=cov)
    assert run.num_rendered > 0
    assert (run.radii > 0).sum() >= 30
    gu = torch.Generator().manual_seed(5)
    up = {"color": torch.randn(3, H, W, generator=gu), "segment": torch.randn(2, H, W, generator=gu),
          "depth": torch.randn(1, H, W, generator=gu), "alpha": torch.randn(1, H, W, generator=gu)}
    og = run.backward(up["color"].numpy(), up["segment"].numpy(), up["depth"].numpy(), up["alpha"].numpy())

    d = lambda t: t.detach().double().clone().requires_grad_(True)
    inp = {"means3D": d(scene.means3D), "means2D": torch.zeros(scene.P, 2, dtype=torch.float64, requires_grad=True),
           "opacities": d(scene.opacities), "segments": d(scene.segments)}
    if colors is not None:
        inp["colors_precomp"] = d(colors)
    else:
        inp["shs"] = d(scene.shs)
    if cov is not None:
        inp["cov3D_precomp"] = d(cov)
    else:
        inp["scales"], inp["rotations"] = d(scene.scales), d(scene.rotations)
    col, dep, alp, seg = restated_render(run, cam, inp, case["deg"], case["bg"], case["mod"])

    # forward: oracle fp32 vs fp64 restatement
    for a, b in ((run.color, col), (run.depth, dep), (run.alpha, alp), (run.segment, seg)):
        np.testing.assert_allclose(a, b.detach().numpy(), rtol=0, atol=2e-5 * max(1.0, float(b.detach().abs().max())))

    loss = (col * up["color"]).sum() + (dep * up["depth"]).sum() + (alp * up["alpha"]).sum() + (seg * up["segment"]).sum()
    keys = [k for k in inp]
    grads = dict(zip(keys, torch.autograd.grad(loss, [inp[k] for k in keys], allow_unused=True)))

    def check(name, ours, ref):
        ref = ref.detach().numpy().reshape(ours.shape)
        scale = max(1e-6, float(np.abs(ref).max()))
        err = float(np.abs(ours - ref).max()) / scale
        assert err < 2e-4, f"{name}: normwise rel err {err:.3e} (max|ref|={scale:.3e})"

    check("dmeans3D", og["dmeans3D"], grads["means3D"])
    check("dmeans2D", og["dmeans2D"][:, :2], grads["means2D"])
    check("dopacity", og["dopacity"], grads["opacities"])
    check("dsegments", og["dsegments"], grads["segments"])
    if colors is not None:
        check("dcolors", og["dcolors"], grads["colors_precomp"])
    else:
        check("dsh", og["dsh"], grads["shs"])
    if cov is not None:
        check("dcov3D", og["dcov3D"], _sym_grad(grads["cov3D_precomp"]))
    else:
        # Reference quirk (kept for parity): computeCov3D backward returns the gradient
        # w.r.t. s = scale_modifier * scale (backward.cu:295-325), i.e. the true
        # dL/dscale divided by scale_modifier.
        check("dscales", og["dscales"], grads["scales"] / case["mod"])
        check("drot", og["drot"], grads["rotations"])


def _sym_grad(g):
    # the restatement reads c[1], c[2], c[4] twice (symmetric matrix); the reference's
    # dL_dcov3D for off-diagonals is the sum of both entries (backward.cu:225-227)
    return g
