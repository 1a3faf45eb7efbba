"""Shared parity machinery: run the HIP path (through the public API) and the CPU
oracle on the same seeded scene, and compare with the tolerances the tests state."""
import math

import numpy as np
import torch


def settings_for(cam, sh_degree, device, bg=(0.0, 0.0, 0.0), scale_modifier=1.0, debug=False):
    from diff_gaussian_rasterization import GaussianRasterizationSettings
    return GaussianRasterizationSettings(
        image_height=int(cam.height), image_width=int(cam.width), tanfovx=cam.tanfovx, tanfovy=cam.tanfovy,
        bg=torch.tensor(bg, dtype=torch.float32, device=device), scale_modifier=scale_modifier,
        viewmatrix=cam.world_view_transform.to(device), projmatrix=cam.full_proj_transform.to(device),
        sh_degree=sh_degree, campos=cam.camera_center.to(device), prefiltered=False, debug=debug)


def upstream_grads(H, W, seed=1, scale=1e-3):
    """Fixed synthetic upstream gradients, N(0,1)*scale."""
    g = torch.Generator().manual_seed(seed)
    mk = lambda c: (torch.randn(c, H, W, generator=g) * scale).contiguous()
    return {"color": mk(3), "depth": mk(1), "alpha": mk(1), "segment": mk(2)}


def run_gsr(scene, cam, device="cuda", bg=(0.0, 0.0, 0.0), scale_modifier=1.0, colors_precomp=None,
            cov3D_precomp=None, use_segments=True, grads=None, want_state=True, sh_degree=None):
    """Forward (+ optional backward) through the drop-in API; returns numpy dicts."""
    from diff_gaussian_rasterization import _C, _RasterizeGaussians
    D = scene.sh_degree if sh_degree is None else sh_degree
    st = settings_for(cam, D, device, bg=bg, scale_modifier=scale_modifier)
    leaf = lambda t: t.detach().to(device).clone().requires_grad_(True)
    means3D = leaf(scene.means3D)
    means2D = torch.zeros_like(means3D, requires_grad=True)
    opac = leaf(scene.opacities)
    segs = leaf(scene.segments) if use_segments else torch.Tensor([])
    if colors_precomp is None:
        shs, cols = leaf(scene.shs), torch.Tensor([])
    else:
        shs, cols = torch.Tensor([]), leaf(colors_precomp)
    if cov3D_precomp is None:
        scales, rots, cov = leaf(scene.scales), leaf(scene.rotations), torch.Tensor([])
    else:
        scales, rots, cov = torch.Tensor([]), torch.Tensor([]), leaf(cov3D_precomp)
    color, radii, depth, alpha, segment = _RasterizeGaussians.apply(
        means3D, means2D, shs, cols, segs, opac, scales, rots, cov, st)
    out = {"color": color, "radii": radii, "depth": depth, "alpha": alpha, "segment": segment}
    res = {k: v.detach().cpu().numpy() for k, v in out.items()}
    if want_state:
        fn = color.grad_fn
        # saved tensors: (colors, segments, means3D, scales, rotations, cov3D, radii, sh, geom, binning, img, alpha)
        saved = fn.saved_tensors
        geom, binning, img = saved[8], saved[9], saved[10]
        P, W, H = scene.P, cam.width, cam.height
        I = _num_rendered(fn)
        res["num_rendered"] = I
        for name in ("tiles_touched", "rec", "clamped", "point_list", "ranges", "n_contrib_tiles", "goff", "bbase",
                     "tile_order", "order"):
            res[name] = _C.debug_state(name, P, W, H, I, geom, binning, img).cpu().numpy()
        res["n_contrib"] = untile_n_contrib(res["n_contrib_tiles"], W, H)
    if grads is not None:
        torch.autograd.backward([color, depth, alpha, segment],
                                [grads["color"].to(device), grads["depth"].to(device), grads["alpha"].to(device),
                                 grads["segment"].to(device)])
        g = {"dmeans3D": means3D.grad, "dmeans2D": means2D.grad, "dopacity": opac.grad}
        if use_segments:
            g["dsegments"] = segs.grad
        if colors_precomp is None:
            g["dsh"] = shs.grad
        else:
            g["dcolors"] = cols.grad
        if cov3D_precomp is None:
            g["dscales"], g["drot"] = scales.grad, rots.grad
        else:
            g["dcov3D"] = cov.grad
        res["grads"] = {k: v.detach().cpu().numpy() for k, v in g.items()}
    torch.cuda.synchronize()
    return res


def _num_rendered(fn):
    # ctx attributes set in forward are readable on the graph node
    return int(fn.num_rendered)


def untile_n_contrib(tiles, W, H):
    """[T,256] tile-major n_contrib in the forward's quadrant layout (entry 64k + lane:
    pixel row 16ty + 8(k>>1) + (lane>>3), col 16tx + 8(k&1) + (lane&7)) -> [H, W]."""
    gx, gy = (W + 15) // 16, (H + 15) // 16
    t = tiles.reshape(gy, gx, 2, 2, 8, 8)        # [ty, tx, kr, kc, r, c]
    img = t.transpose(0, 2, 4, 1, 3, 5).reshape(gy * 16, gx * 16)
    return img[:H, :W]


def run_oracle(oracle_mod, scene, cam, bg=(0.0, 0.0, 0.0), scale_modifier=1.0, colors_precomp=None,
               cov3D_precomp=None, use_segments=True, grads=None, sh_degree=None):
    run = oracle_mod.run_scene(scene, cam, bg=bg, scale_modifier=scale_modifier, colors_precomp=colors_precomp,
                               cov3D_precomp=cov3D_precomp,
                               segments="scene" if use_segments else None, sh_degree=sh_degree)
    res = {"color": run.color, "depth": run.depth, "alpha": run.alpha, "segment": run.segment,
           "radii": run.radii, "num_rendered": run.num_rendered}
    for k in ("tiles_touched", "point_list", "ranges", "n_contrib", "means2D", "conic_opacity", "depths", "rgb",
              "clamped"):
        res[k] = run.get(k)
    res["n_contrib"] = res["n_contrib"].reshape(cam.height, cam.width)
    if grads is not None:
        g = run.backward(grads["color"].numpy(), grads["segment"].numpy(), grads["depth"].numpy(),
                         grads["alpha"].numpy())
        res["grads"] = g
    res["_run"] = run
    return res


def tol_report(a, b, scale_floor=1.0):
    """max |a-b| / max(scale_floor, |b|) elementwise (the SURVEY s7 tolerance form)."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    if a.size == 0:
        return 0.0
    return float(np.max(np.abs(a - b) / np.maximum(scale_floor, np.abs(b))))


def reference_noise(oracle_mod, run, grads, ref_grads):
    """Per tensor: max |acc32 - exact| / max|exact| -- how far the reference's own fp32
    atomicAdd accumulation (the oracle summing in one fixed fp32 order, set_acc32) moves each
    gradient from the exact sums the oracle reports.  `run` is run_oracle's "_run"."""
    oracle_mod.set_acc32(True)
    try:
        g32 = run.backward(grads["color"].numpy(), grads["segment"].numpy(), grads["depth"].numpy(),
                           grads["alpha"].numpy())
    finally:
        oracle_mod.set_acc32(False)
    out = {}
    for k, ref in ref_grads.items():
        a, b = g32[k].astype(np.float64), ref.astype(np.float64)
        if k == "dmeans2D":
            a, b = a[:, :2], b[:, :2]
        m = float(np.abs(b).max()) if b.size else 0.0
        out[k] = float(np.abs(a - b).max() / m) if m > 0 else 0.0
    return out
