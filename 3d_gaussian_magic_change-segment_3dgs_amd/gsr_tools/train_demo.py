"""A minimal training loop over the MI355X path: gsr_train.GaussianModel +
diff_gaussian_rasterization + GaussianAdam + on-device densification, in the
shape of the reference's train.py:80-190 (render -> L1 loss -> backward ->
densification statistics -> densify_and_prune every `densify_interval` -> Adam
step).  Used by tests/test_gpu_training.py as the end-to-end check of the SURVEY
s8f components working together; not a replacement for train.py's I/O, logging
or depth / SSIM losses (out of scope).

`render` mirrors gaussian_renderer/__init__.py:render (the non-bbox branch,
:296-391): screen-space dummy with retain_grad, settings from the camera, the
rasterizer called with the model's activated tensors, depth / (max + 1e-5).
"""
import math

import torch

from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer


def render(cam, pc, bg_color, scaling_modifier=1.0, debug=False):
    dev = pc.device
    screenspace_points = torch.zeros_like(pc.get_xyz, dtype=pc.get_xyz.dtype, requires_grad=True, device=dev) + 0
    if screenspace_points.requires_grad:  # (the reference wraps this in try/except for no_grad renders)
        screenspace_points.retain_grad()
    raster_settings = GaussianRasterizationSettings(
        image_height=int(cam.height), image_width=int(cam.width), tanfovx=math.tan(cam.FoVx * 0.5),
        tanfovy=math.tan(cam.FoVy * 0.5), bg=bg_color, scale_modifier=scaling_modifier,
        viewmatrix=cam.world_view_transform.to(dev), projmatrix=cam.full_proj_transform.to(dev),
        sh_degree=pc.active_sh_degree, campos=cam.camera_center.to(dev), prefiltered=False, debug=debug)
    rasterizer = GaussianRasterizer(raster_settings=raster_settings)
    rendered_image, radii, depth, alpha, rendered_segment = rasterizer(
        means3D=pc.get_xyz, means2D=screenspace_points, opacities=pc.get_opacity, shs=pc.get_features,
        colors_precomp=None, segments=pc.get_segment, scales=pc.get_scaling, rotations=pc.get_rotation,
        cov3D_precomp=None)
    depth = depth / (depth.max() + 1e-5)
    return {"render": rendered_image, "viewspace_points": screenspace_points, "visibility_filter": radii > 0,
            "radii": radii, "depth": depth, "alpha": alpha, "segment": rendered_segment}


class OptArgs:
    """OptimizationParams defaults (arguments/__init__.py:90-113) used by the loop."""
    position_lr_init, position_lr_final, position_lr_delay_mult, position_lr_max_steps = 0.00016, 0.0000016, 0.01, 30000
    feature_lr, opacity_lr, segment_lr, scaling_lr, rotation_lr = 0.0025, 0.05, 0.05, 0.005, 0.001
    percent_dense = 0.01
    densification_interval, densify_from_iter, densify_until_iter = 100, 500, 15000
    densify_grad_threshold, opacity_reset_interval = 0.0002, 3000


def train(gaussians, cams, targets, iters, opt=OptArgs, bg=None, extent=1.0, log=None, generator=None):
    """Run `iters` iterations over the cameras in order; returns the per-iteration L1 losses."""
    dev = gaussians.device
    bg = torch.zeros(3, device=dev) if bg is None else bg
    gaussians.training_setup(opt)
    losses = []
    for it in range(1, iters + 1):
        gaussians.update_learning_rate(it)
        cam, gt = cams[(it - 1) % len(cams)], targets[(it - 1) % len(cams)]
        pkg = render(cam, gaussians, bg)
        loss = (pkg["render"] - gt).abs().mean()
        loss.backward()
        losses.append(float(loss.detach()))
        with torch.no_grad():
            if it < opt.densify_until_iter:
                gaussians.update_densification_stats(pkg["viewspace_points"], pkg["radii"])
                if it > opt.densify_from_iter and it % opt.densification_interval == 0:
                    size_threshold = 20 if it > opt.opacity_reset_interval else None
                    gaussians.densify_and_prune(opt.densify_grad_threshold, 0.005, extent, size_threshold,
                                                generator=generator)
                if it % opt.opacity_reset_interval == 0:
                    gaussians.reset_opacity()
            gaussians.optimizer.step()
            gaussians.optimizer.zero_grad(set_to_none=True)
        if log is not None:
            log(it, losses[-1], gaussians.num_points)
    return losses
