#
# Portions of this file (the public API surface: GaussianRasterizationSettings,
# GaussianRasterizer, rasterize_gaussians, _RasterizeGaussians -- their argument
# tuples, validation messages and debug snapshot handling) follow
# submodules_local/diff-gaussian-rasterization/diff_gaussian_rasterization/__init__.py
# of the reference, which carries this notice:
#
# Copyright (C) 2023, Inria
# GRAPHDECO research group, https://team.inria.fr/graphdeco
# All rights reserved.
#
# This software is free for non-commercial, research and evaluation use
# under the terms of the LICENSE.md file.
#
# For inquiries contact  george.drettakis@inria.fr
#
"""diff_gaussian_rasterization -- MI355X-native drop-in for the reference's
differentiable Gaussian rasterizer (DGR/diff_gaussian_rasterization/__init__.py).

Public API identical to the reference: GaussianRasterizationSettings (:168-180),
GaussianRasterizer with forward/markVisible (:182-235), rasterize_gaussians
(:21-44) and the autograd function _RasterizeGaussians (:46-166), so that
gaussian_renderer/__init__.py imports and calls it unchanged.  The compute path
is libgsr.so (hand-written HIP for gfx950) through the ctypes module `_C`.
"""
import contextlib
import os
import threading
from typing import NamedTuple

import torch
import torch.nn as nn

from . import _C

__all__ = ["GaussianRasterizationSettings", "GaussianRasterizer", "rasterize_gaussians",
           "rasterize_gaussians_multiview", "defer_sh_gradients"]

# Process-wide, not thread-local: autograd runs the backward of GPU tensors on its own
# device thread, not on the thread that entered the context.
_SINKS = []
_SINKS_LOCK = threading.Lock()


class defer_sh_gradients:
    """Context manager for view-parallel training (gsr_tools.dp.ShExchange): backward
    passes run inside it leave the SH gradient to a later exchange.  They write
    each view's SH exchange rows (include/gsr.h gsr_backward_multiview_deferred_sh)
    to a buffer obtained from `sink.sh_rows(B, P, device)` and report the call with
    `sink.record(...)`; the returned dsh is NOT written until the sink runs
    _C.sh_backward (every other gradient, dmeans3D included, is complete; a single view
    goes through gsr_backward_deferred_sh, several through the multi-view call).  Calls without SH
    coefficients (colors_precomp) are unaffected.  The context is process-wide (the
    autograd engine runs GPU backwards on its own threads).  An extension of the
    reference API."""

    def __init__(self, sink):
        self.sink = sink

    def __enter__(self):
        with _SINKS_LOCK:
            _SINKS.append(self.sink)
            _sinks_changed()
        return self.sink

    def __exit__(self, *exc):
        with _SINKS_LOCK:
            _SINKS.remove(self.sink)
            _sinks_changed()
        return False


def _sinks_changed():
    # the C++ autograd route (_C._HOST_AUTOGRAD) checks the count at backward time
    if _C._HOST_AUTOGRAD is not None:
        _C._HOST_AUTOGRAD.set_sinks(len(_SINKS))


# the multi-view forward's side stream per device (GSR_MV_STREAMS=0: one stream)
_MV_STREAMS = os.environ.get("GSR_MV_STREAMS", "1") != "0"
_VIEW_STREAMS = {}


# streams the multi-view forward deals its views over (the caller's + MV_FWD_STREAMS - 1 side ones)
_MV_FWD_STREAMS = max(2, int(os.environ.get("GSR_MV_FWD_STREAMS", "2")))


def _view_streams(device, n):
    sts = _VIEW_STREAMS.setdefault(device, [])
    while len(sts) < n:
        sts.append(torch.cuda.Stream(device=device))
    return sts[:n]


def _sh_sink():
    with _SINKS_LOCK:
        return _SINKS[-1] if _SINKS else None


def _backward_views(views, means3D, colors_precomp, segments, scales, rotations, scale_modifier, cov3Ds_precomp,
                    sh, sh_degree, debug):
    """Multi-view backward, deferred-SH when a defer_sh_gradients sink is active."""
    sink = _sh_sink()
    rows = None
    if sink is not None and isinstance(sh, torch.Tensor) and sh.numel() > 0:
        rows = sink.sh_rows(len(views), int(means3D.size(0)), means3D.device)
    out, d2 = _C.rasterize_gaussians_backward_multiview(views, means3D, colors_precomp, segments, scales, rotations,
                                                        scale_modifier, cov3Ds_precomp, sh, sh_degree, debug,
                                                        sh_rows=rows)
    if rows is not None:
        _, _, _, g_means3D, _, g_sh, _, _, _ = out
        sink.record(rows, len(views), means3D, sh, sh_degree, g_sh, g_means3D,
                    inputs=tuple(t for t in (segments, scales, rotations) if isinstance(t, torch.Tensor)))
    return out, d2


def cpu_deep_copy_tuple(input_tuple):
    copied_tensors = [item.cpu().clone() if isinstance(item, torch.Tensor) else item for item in input_tuple]
    return tuple(copied_tensors)


def rasterize_gaussians(
    means3D,
    means2D,
    sh,
    colors_precomp,
    segments,
    opacities,
    scales,
    rotations,
    cov3Ds_precomp,
    raster_settings,
):
    s = raster_settings
    if _C._HOST_AUTOGRAD is not None and not s.debug and not _SINKS:
        # the same autograd function in C++ (csrc/host_ext.cpp RasterizeFn): same outputs, saved
        # state and gradients, without autograd's Python hops.  Debug mode (snapshot dumps) and
        # forwards inside defer_sh_gradients take _RasterizeGaussians.
        device = means3D.device
        *out, num_rendered = _C._HOST_AUTOGRAD.rasterize(
            means3D, means2D, sh, colors_precomp, segments, opacities, scales, rotations, cov3Ds_precomp, s.bg,
            s.viewmatrix, s.projmatrix, s.campos, float(s.scale_modifier), float(s.tanfovx), float(s.tanfovy),
            int(s.image_height), int(s.image_width), int(s.sh_degree), bool(s.prefiltered), _C._guess(device))
        if means3D.size(0) > 0:
            _C._record(device, num_rendered)
        return tuple(out)
    return _RasterizeGaussians.apply(
        means3D,
        means2D,
        sh,
        colors_precomp,
        segments,
        opacities,
        scales,
        rotations,
        cov3Ds_precomp,
        raster_settings,
    )


class _RasterizeGaussians(torch.autograd.Function):
    @staticmethod
    def forward(ctx, means3D, means2D, sh, colors_precomp, segments, opacities, scales, rotations, cov3Ds_precomp,
                raster_settings):
        # Same argument order as the reference's C++ entry point (rasterize_points.h:18-39)
        args = (
            raster_settings.bg,
            means3D,
            colors_precomp,
            segments,
            opacities,
            scales,
            rotations,
            raster_settings.scale_modifier,
            cov3Ds_precomp,
            raster_settings.viewmatrix,
            raster_settings.projmatrix,
            raster_settings.tanfovx,
            raster_settings.tanfovy,
            raster_settings.image_height,
            raster_settings.image_width,
            sh,
            raster_settings.sh_degree,
            raster_settings.campos,
            raster_settings.prefiltered,
            raster_settings.debug,
        )
        if raster_settings.debug:
            cpu_args = cpu_deep_copy_tuple(args)  # copy before they can be corrupted
            try:
                out = _C.rasterize_gaussians(*args)
            except Exception as ex:
                torch.save(cpu_args, "snapshot_fw.dump")
                print("\nAn error occured in forward. Please forward snapshot_fw.dump for debugging.")
                raise ex
        else:
            out = _C.rasterize_gaussians(*args)
        num_rendered, color, depth, segment, alpha, radii, geomBuffer, binningBuffer, imgBuffer = out

        ctx.raster_settings = raster_settings
        ctx.num_rendered = num_rendered
        ctx.save_for_backward(colors_precomp, segments, means3D, scales, rotations, cov3Ds_precomp, radii, sh,
                              geomBuffer, binningBuffer, imgBuffer, alpha)
        ctx.mark_non_differentiable(radii)
        # No zero-filled stand-ins for outputs without a gradient (radii, or an image the
        # loss does not use): the backward reads a missing image gradient as zeros.
        ctx.set_materialize_grads(False)
        return color, radii, depth, alpha, segment

    @staticmethod
    def backward(ctx, grad_color, grad_radii, grad_depth, grad_alpha, grad_segment):
        num_rendered = ctx.num_rendered
        raster_settings = ctx.raster_settings
        (colors_precomp, segments, means3D, scales, rotations, cov3Ds_precomp, radii, sh, geomBuffer, binningBuffer,
         imgBuffer, alpha) = ctx.saved_tensors
        args = (raster_settings.bg,
                means3D,
                radii,
                colors_precomp,
                segments,
                scales,
                rotations,
                raster_settings.scale_modifier,
                cov3Ds_precomp,
                raster_settings.viewmatrix,
                raster_settings.projmatrix,
                raster_settings.tanfovx,
                raster_settings.tanfovy,
                grad_color,
                grad_segment,
                grad_depth,
                grad_alpha,
                sh,
                raster_settings.sh_degree,
                raster_settings.campos,
                geomBuffer,
                num_rendered,
                binningBuffer,
                imgBuffer,
                alpha,
                raster_settings.debug)
        sink = _sh_sink() if sh.numel() > 0 else None
        if sink is not None:
            out = _sink_backward(sink, args)
        elif raster_settings.debug:
            cpu_args = cpu_deep_copy_tuple(args)
            try:
                out = _C.rasterize_gaussians_backward(*args)
            except Exception as ex:
                torch.save(cpu_args, "snapshot_bw.dump")
                print("\nAn error occured in backward. Writing snapshot_bw.dump for debugging.\n")
                raise ex
        else:
            out = _C.rasterize_gaussians_backward(*args)
        (grad_means2D, grad_colors_precomp, grad_opacities, grad_means3D, grad_cov3Ds_precomp, grad_sh, grad_scales,
         grad_rotations, grad_segments) = out

        grads = (
            grad_means3D,
            grad_means2D,
            grad_sh,
            grad_colors_precomp,
            grad_segments,
            grad_opacities,
            grad_scales,
            grad_rotations,
            grad_cov3Ds_precomp,
            None,
        )
        return _finish_grads(ctx, grads)


def _sink_backward(sink, args):
    """Deferred SH (view-parallel exchange): the single-view backward writes this view's exchange
    rows instead of dsh (include/gsr.h gsr_backward_deferred_sh).  args: _C.rasterize_gaussians_backward's."""
    means3D, segments, scales, rotations, sh, sh_degree = args[1], args[4], args[5], args[6], args[17], args[18]
    rows = sink.sh_rows(1, int(means3D.size(0)), means3D.device)
    out = _C.rasterize_gaussians_backward(*args, sh_rows=rows)
    sink.record(rows, 1, means3D, sh, sh_degree, out[5], out[3],
                inputs=tuple(t for t in (segments, scales, rotations) if isinstance(t, torch.Tensor)))
    return out


def _cpp_sink_backward(*args):
    """Backward of the C++ autograd route that found a defer_sh_gradients sink active (the forward
    ran outside the context): the sink's route, as _RasterizeGaussians.backward takes it.  args:
    _C.rasterize_gaussians_backward's without debug."""
    sink = _sh_sink()
    args = args + (False,)
    return _sink_backward(sink, args) if sink is not None else _C.rasterize_gaussians_backward(*args)


if _C._HOST_AUTOGRAD is not None:
    _C._HOST_AUTOGRAD.set_sink_backward(_cpp_sink_backward)


def rasterize_gaussians_multiview(means3D, means2D_list, sh, colors_precomp, segments, opacities, scales, rotations,
                                  cov3Ds_precomp, raster_settings_list):
    """Several views of the same Gaussians (the batch of a view-parallel trainer step):
    per view the forward of rasterize_gaussians, and ONE backward that sums the
    parameter gradients over the views (include/gsr.h gsr_backward_multiview; the
    per-Gaussian work and parameter traffic happen once per batch).  means2D_list
    holds one screen-space dummy per view (its .grad is that view's gradient, for
    the densification statistics).  Returns a list of (color, radii, depth, alpha,
    segment) per view.  Same inputs and conventions as rasterize_gaussians; an
    extension of the reference API (which renders one view per call)."""
    B = len(raster_settings_list)
    if B != len(means2D_list):
        raise ValueError("one means2D per view")
    outs = _RasterizeGaussiansMultiview.apply(means3D, sh, colors_precomp, segments, opacities, scales, rotations,
                                              cov3Ds_precomp, tuple(raster_settings_list), *means2D_list)
    return [tuple(outs[5 * v:5 * v + 5]) for v in range(B)]


class _RasterizeGaussiansMultiview(torch.autograd.Function):
    @staticmethod
    def forward(ctx, means3D, sh, colors_precomp, segments, opacities, scales, rotations, cov3Ds_precomp,
                settings_list, *means2D_list):
        # Views alternate between the caller's stream and a side stream, so that view v+1's
        # preprocess and binning (short, latency-bound launches) run beside view v's render
        # tail; the caller's stream then waits for the side stream.  Tensors made on the side
        # stream are recorded on the caller's (caching-allocator rule for cross-stream use).
        outs, views = [], []
        dev = means3D.device
        main = torch.cuda.current_stream(dev) if means3D.is_cuda else None
        multi = (main is not None and len(settings_list) > 1 and _MV_STREAMS
                 and not any(rs.debug for rs in settings_list))
        # view v runs on stream v % K: the caller's (0) or a side stream
        sides = _view_streams(dev, min(_MV_FWD_STREAMS, len(settings_list)) - 1) if multi else []
        for sd in sides:
            sd.wait_stream(main)
        vstream = lambda v: sides[v % (len(sides) + 1) - 1] if sides and v % (len(sides) + 1) else None
        # Every view's forward is launched before any view's num_rendered is waited for
        # (rasterize_gaussians_begin / _end: gsr_forward_deferred), so that the host's launches
        # are not gated on each view's binning: both streams stay fed.
        handles = []
        try:
            for v, rs in enumerate(settings_list):
                sv = vstream(v)
                with torch.cuda.stream(sv) if sv is not None else contextlib.nullcontext():
                    handles.append(_C.rasterize_gaussians_begin(
                        rs.bg, means3D, colors_precomp, segments, opacities, scales, rotations, rs.scale_modifier,
                        cov3Ds_precomp, rs.viewmatrix, rs.projmatrix, rs.tanfovx, rs.tanfovy, rs.image_height,
                        rs.image_width, sh, rs.sh_degree, rs.campos, rs.prefiltered, rs.debug))
            for v, rs in enumerate(settings_list):
                sv = vstream(v)
                h, handles[v] = handles[v], None   # ended (its ticket freed) even if _end raises
                with torch.cuda.stream(sv) if sv is not None else contextlib.nullcontext():
                    out = _C.rasterize_gaussians_end(h)
                num_rendered, color, depth, segment, alpha, radii, geom, binning, img = out
                if sv is not None:
                    for t in (color, depth, segment, alpha, radii, geom, binning, img):
                        if t.is_cuda and t.numel() > 0:
                            t.record_stream(main)
                views.append((num_rendered, radii, geom, binning, img, alpha))
                ctx.mark_non_differentiable(radii)
                outs += [color, radii, depth, alpha, segment]
        except BaseException:
            # every started forward that has not been ended is ended now (tickets are per-thread
            # pinned slots, GSR_MAX_DEFERRED of them: a leaked one fails every later batch)
            for v, h in enumerate(handles):
                if h is None:
                    continue
                try:
                    sv = vstream(v)
                    with torch.cuda.stream(sv) if sv is not None else contextlib.nullcontext():
                        _C.rasterize_gaussians_end(h)
                except Exception:
                    pass
            raise
        finally:
            for sd in sides:
                main.wait_stream(sd)
        ctx.settings_list = settings_list
        ctx.views = views
        ctx.save_for_backward(colors_precomp, segments, means3D, scales, rotations, cov3Ds_precomp, sh)
        ctx.set_materialize_grads(False)
        return tuple(outs)

    @staticmethod
    def backward(ctx, *grad_outputs):
        colors_precomp, segments, means3D, scales, rotations, cov3Ds_precomp, sh = ctx.saved_tensors
        rs0 = ctx.settings_list[0]
        views = []
        for v, (rs, st) in enumerate(zip(ctx.settings_list, ctx.views)):
            num_rendered, radii, geom, binning, img, alpha = st
            gc, _, gd, ga, gs = grad_outputs[5 * v:5 * v + 5]
            views.append({"bg": rs.bg, "viewmatrix": rs.viewmatrix, "projmatrix": rs.projmatrix,
                          "tanfovx": rs.tanfovx, "tanfovy": rs.tanfovy, "image_height": rs.image_height,
                          "image_width": rs.image_width, "campos": rs.campos, "radii": radii, "geom": geom,
                          "binning": binning, "img": img, "num_rendered": num_rendered, "alpha": alpha,
                          "dL_dcolor": gc, "dL_dsegment": gs, "dL_ddepth": gd, "dL_dalpha": ga})
        (_, g_colors, g_opacities, g_means3D, g_cov3D, g_sh, g_scales, g_rot, g_segments), d2 = \
            _backward_views(views, means3D, colors_precomp, segments, scales, rotations, rs0.scale_modifier,
                            cov3Ds_precomp, sh, rs0.sh_degree, rs0.debug)
        ctx.views = None
        return _finish_grads(ctx, (g_means3D, g_sh, g_colors, g_segments, g_opacities, g_scales, g_rot, g_cov3D,
                                   None, *d2))


def _finish_grads(ctx, grads):
    """Gradients handed to autograd: None where the input needs none (the backward's
    zero placeholders for absent inputs are stride-0 views of one cached zero), and a
    real zero tensor where an input that needs a gradient got such a placeholder, so that
    hooks or in-place ops on .grad never see aliased memory (rasterize_points.cu:166-177
    returns torch.zeros tensors)."""
    out = []
    for need, g in zip(ctx.needs_input_grad, grads):
        if g is None or not need:
            out.append(None)
        elif g.numel() > 0 and 0 in g.stride():
            out.append(torch.zeros(g.shape, dtype=g.dtype, device=g.device))
        else:
            out.append(g)
    return tuple(out)


class GaussianRasterizationSettings(NamedTuple):
    image_height: int
    image_width: int
    tanfovx: float
    tanfovy: float
    bg: torch.Tensor
    scale_modifier: float
    viewmatrix: torch.Tensor
    projmatrix: torch.Tensor
    sh_degree: int
    campos: torch.Tensor
    prefiltered: bool
    debug: bool


class GaussianRasterizer(nn.Module):
    def __init__(self, raster_settings):
        super().__init__()
        self.raster_settings = raster_settings

    def markVisible(self, positions):
        # Mark visible points (based on frustum culling for camera) with a boolean
        with torch.no_grad():
            raster_settings = self.raster_settings
            visible = _C.mark_visible(
                positions,
                raster_settings.viewmatrix,
                raster_settings.projmatrix)
        return visible

    def forward(self, means3D, means2D, opacities, shs=None, colors_precomp=None, segments=None, scales=None,
                rotations=None, cov3D_precomp=None):
        raster_settings = self.raster_settings

        if (shs is None and colors_precomp is None) or (shs is not None and colors_precomp is not None):
            raise Exception('Please provide excatly one of either SHs or precomputed colors!')

        if ((scales is None or rotations is None) and cov3D_precomp is None) or (
                (scales is not None or rotations is not None) and cov3D_precomp is not None):
            raise Exception('Please provide exactly one of either scale/rotation pair or precomputed 3D covariance!')

        if shs is None:
            shs = torch.Tensor([])
        if colors_precomp is None:
            colors_precomp = torch.Tensor([])

        if segments is None:
            segments = torch.Tensor([])

        if scales is None:
            scales = torch.Tensor([])
        if rotations is None:
            rotations = torch.Tensor([])
        if cov3D_precomp is None:
            cov3D_precomp = torch.Tensor([])

        # Invoke the HIP rasterization routine
        return rasterize_gaussians(
            means3D,
            means2D,
            shs,
            colors_precomp,
            segments,
            opacities,
            scales,
            rotations,
            cov3D_precomp,
            raster_settings,
        )
