"""The drop-in API on the GPU, called exactly the way the reference's
gaussian_renderer/__init__.py:314-373 calls it."""
import os

import numpy as np
import pytest
import torch

import harness as Hn
from gsr_tools.scene import synthetic_scene, orbit_camera

pytestmark = pytest.mark.gpu


def _renderer_style_call(scene, cam, debug=False):
    """Mirror of render() in gaussian_renderer/__init__.py (activations on parameters,
    screenspace_points with retain_grad, kwargs call, 5 outputs, depth/max)."""
    from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer
    dev = "cuda"
    xyz = torch.nn.Parameter(scene.means3D.to(dev))
    opacity_raw = torch.nn.Parameter(torch.logit(scene.opacities.to(dev)))
    seg_raw = torch.nn.Parameter(torch.logit(scene.segments.to(dev)))
    scale_raw = torch.nn.Parameter(torch.log(scene.scales.to(dev)))
    rot_raw = torch.nn.Parameter(scene.rotations.to(dev) * 2.0)
    feats = torch.nn.Parameter(scene.shs.to(dev))
    screenspace_points = torch.zeros_like(xyz, dtype=xyz.dtype, requires_grad=True, device="cuda") + 0
    screenspace_points.retain_grad()
    raster_settings = GaussianRasterizationSettings(
        image_height=int(cam.height), image_width=int(cam.width), tanfovx=cam.tanfovx, tanfovy=cam.tanfovy,
        bg=torch.tensor([0.0, 0.0, 0.0], device=dev), scale_modifier=1.0,
        viewmatrix=cam.world_view_transform.to(dev), projmatrix=cam.full_proj_transform.to(dev),
        sh_degree=scene.sh_degree, campos=cam.camera_center.to(dev), prefiltered=False, debug=debug)
    rasterizer = GaussianRasterizer(raster_settings=raster_settings)
    rendered_image, radii, depth, alpha, rendered_segment = rasterizer(
        means3D=xyz, means2D=screenspace_points, opacities=torch.sigmoid(opacity_raw), shs=feats,
        colors_precomp=None, segments=torch.sigmoid(seg_raw), scales=torch.exp(scale_raw),
        rotations=torch.nn.functional.normalize(rot_raw), cov3D_precomp=None)
    depth = depth / (depth.max() + 1e-5)
    loss = rendered_image.mean() + depth.mean() + alpha.mean() + rendered_segment.mean()
    loss.backward()
    params = dict(xyz=xyz, opacity=opacity_raw, seg=seg_raw, scale=scale_raw, rot=rot_raw, feats=feats)
    return rendered_image, radii, screenspace_points, params, rasterizer


def test_renderer_style_call_and_grads(gpu_available):
    scene = synthetic_scene(5000, sh_degree=3, seed=21)
    cam = orbit_camera(4, 160, 120, 150.0)
    img, radii, ssp, params, _ = _renderer_style_call(scene, cam)
    assert img.shape == (3, 120, 160) and radii.dtype == torch.int32
    vis = radii > 0
    assert int(vis.sum()) > 1000
    assert ssp.grad is not None and torch.isfinite(ssp.grad).all()
    assert float(ssp.grad[vis, :2].abs().sum()) > 0 and float(ssp.grad[~vis].abs().sum()) == 0
    for n, p in params.items():
        assert p.grad is not None and torch.isfinite(p.grad).all(), n
        assert float(p.grad.abs().sum()) > 0, n


def test_debug_mode_matches(gpu_available):
    scene = synthetic_scene(3000, sh_degree=2, seed=22)
    cam = orbit_camera(5, 128, 96, 120.0)
    a = _renderer_style_call(scene, cam, debug=False)
    b = _renderer_style_call(scene, cam, debug=True)
    assert torch.equal(a[0], b[0])
    for n in a[3]:
        assert torch.equal(a[3][n].grad, b[3][n].grad), n


def test_mark_visible_matches_oracle(gpu_available, oracle_mod):
    scene = synthetic_scene(4000, sh_degree=0, seed=23, extent=4.0)
    cam = orbit_camera(1, 64, 64, 60.0)
    *_, rasterizer = _renderer_style_call(synthetic_scene(10, sh_degree=0, seed=1), cam)
    vis = rasterizer.markVisible(scene.means3D.cuda()).cpu().numpy()
    ref = oracle_mod.mark_visible(scene.means3D, cam.world_view_transform.numpy())
    np.testing.assert_array_equal(vis, ref)
    assert 0 < vis.sum() < len(vis)


def test_argument_validation(gpu_available):
    from diff_gaussian_rasterization import GaussianRasterizer
    cam = orbit_camera(0, 32, 32, 30.0)
    st = Hn.settings_for(cam, 0, "cuda")
    r = GaussianRasterizer(st)
    m = torch.zeros(4, 3, device="cuda")
    o = torch.ones(4, 1, device="cuda")
    with pytest.raises(Exception, match="excatly one of either SHs"):  # reference's own spelling (:203)
        r(means3D=m, means2D=m, opacities=o, scales=m, rotations=torch.ones(4, 4, device="cuda"))
    with pytest.raises(Exception, match="scale/rotation"):
        r(means3D=m, means2D=m, opacities=o, shs=torch.ones(4, 1, 3, device="cuda"), scales=m)
    with pytest.raises(RuntimeError, match="means3D must have dimensions"):
        r(means3D=torch.zeros(4, 2, device="cuda"), means2D=m, opacities=o, shs=torch.ones(4, 1, 3, device="cuda"),
          scales=m, rotations=torch.ones(4, 4, device="cuda"))


def test_side_stream_matches_default_stream(gpu_available):
    scene = synthetic_scene(4000, sh_degree=3, seed=24)
    cam = orbit_camera(6, 128, 128, 120.0)
    a = Hn.run_gsr(scene, cam, want_state=False)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        b = Hn.run_gsr(scene, cam, want_state=False)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(a["color"], b["color"])


def test_native_library_is_in_tree(gpu_available):
    """The HIP path is libgsr.so from this repository (no site-packages copy, no fallback)."""
    from diff_gaussian_rasterization import _C
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    assert os.path.realpath(_C.LIB_PATH).startswith(os.path.realpath(root))
    maps = open("/proc/self/maps").read()
    assert os.path.realpath(_C.LIB_PATH) in maps


def test_loss_on_colour_only(gpu_available):
    """Images the loss does not use get no gradient (None in backward): gsr reads them
    as zeros, so the result equals passing explicit zero upstream gradients."""
    from diff_gaussian_rasterization import _RasterizeGaussians
    scene = synthetic_scene(4000, sh_degree=2, seed=23)
    cam = orbit_camera(5, 128, 96, 140.0)
    st = Hn.settings_for(cam, scene.sh_degree, "cuda")
    E = torch.Tensor([])

    def run(explicit_zeros):
        leaf = lambda t: t.detach().to("cuda").clone().requires_grad_(True)
        ins = [leaf(scene.means3D), torch.zeros(scene.P, 3, device="cuda", requires_grad=True), leaf(scene.shs),
               E, leaf(scene.segments), leaf(scene.opacities), leaf(scene.scales), leaf(scene.rotations), E]
        color, radii, depth, alpha, segment = _RasterizeGaussians.apply(*ins, st)
        g = torch.full_like(color, 1e-3)
        if explicit_zeros:
            torch.autograd.backward([color, depth, alpha, segment],
                                    [g, torch.zeros_like(depth), torch.zeros_like(alpha), torch.zeros_like(segment)])
        else:
            torch.autograd.backward([color], [g])
        return [t.grad for t in ins if isinstance(t, torch.Tensor) and t.requires_grad]

    for a, b in zip(run(False), run(True)):
        torch.testing.assert_close(a, b, rtol=0, atol=0)


def _outputs_and_grads(scene, cam):
    img, radii, ssp, params, _ = _renderer_style_call(scene, cam)
    out = {"img": img.detach().clone(), "radii": radii.clone(), "ssp": ssp.grad.clone()}
    out.update({n: p.grad.clone() for n, p in params.items()})
    return out


def test_speculative_stage_b_matches_exact(gpu_available):
    """gsr_forward with a binning-capacity guess launches stage B before num_rendered
    reaches the host (gsr.h).  It must give bit-identical images and gradients to the
    exact path, both when the guess holds and when it is too small (GSR_NEED_BINNING ->
    stage B re-run with the exact buffer)."""
    from diff_gaussian_rasterization import _C
    small = synthetic_scene(800, sh_degree=3, seed=31)
    big = synthetic_scene(6000, sh_degree=3, seed=32)
    cam = orbit_camera(2, 176, 128, 160.0)
    saved = dict(_C._last_rendered)
    try:
        _C.set_option("speculate", 0)
        _C._last_rendered.clear()
        ref_big = _outputs_and_grads(big, cam)     # exact path (no guess)
        ref_small = _outputs_and_grads(small, cam)  # guess buffer from big, stage B after the sync
        _C.set_option("speculate", 1)
        _C._last_rendered.clear()
        _outputs_and_grads(small, cam)             # sets the guess from the small scene
        spec_big = _outputs_and_grads(big, cam)    # guess too small: NEED_BINNING fallback
        spec_big2 = _outputs_and_grads(big, cam)   # guess from big: speculative stage B holds
        spec_small = _outputs_and_grads(small, cam)  # capacity far above num_rendered
    finally:
        _C.set_option("speculate", 1)
        _C._last_rendered.clear()
        _C._last_rendered.update(saved)
    for got, ref in ((spec_big, ref_big), (spec_big2, ref_big), (spec_small, ref_small)):
        for k in ref:
            assert torch.equal(got[k], ref[k]), k


def test_stream_copy_reference_kernel(gpu_available):
    """gsr_stream_copy (bench.py's measured HBM copy rate) moves the bytes exactly for every
    float4-per-thread variant, including a tail that is not a multiple of the block, and
    rejects bad arguments."""
    import torch
    from diff_gaussian_rasterization import _C
    n = 1_000_003 * 4  # floats: 16-B multiple, not a multiple of 256 threads * 4 float4
    src = torch.randn(n, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    for u in (1, 2, 4):
        dst = torch.full_like(src, float("nan"))
        assert _C._lib.gsr_stream_copy(src.data_ptr(), dst.data_ptr(), n * 4, u, st) == 0
        torch.cuda.synchronize()
        assert torch.equal(src, dst)
    dst = torch.empty_like(src)
    assert _C._lib.gsr_stream_copy(src.data_ptr(), dst.data_ptr(), 12, 1, st) != 0  # not a multiple of 16
    assert _C._lib.gsr_stream_copy(src.data_ptr(), dst.data_ptr(), 16, 3, st) != 0  # bad variant


def test_absent_input_gradients_are_not_aliased_views(gpu_available):
    """the backward's zero placeholders for absent inputs (stride-0 views of one
    cached zero) never reach autograd.  Inputs that need no gradient get None; a leaf whose
    gradient is such a placeholder would get a real zero tensor, so in-place ops on .grad
    work (the reference returns torch.zeros tensors, rasterize_points.cu:166-177)."""
    import harness as Hn
    from diff_gaussian_rasterization import _RasterizeGaussians
    from gsr_tools.scene import synthetic_scene, orbit_camera
    scene = synthetic_scene(2000, sh_degree=3, seed=71)
    cam = orbit_camera(0, 96, 64, 80.0)
    st = Hn.settings_for(cam, 3, "cuda")
    L = lambda t: t.detach().cuda().clone().requires_grad_(True)
    means3D, opac, segs = L(scene.means3D), L(scene.opacities), L(scene.segments)
    cols = L(torch.rand(scene.P, 3))
    g = torch.Generator().manual_seed(2)
    A = torch.randn(scene.P, 3, 3, generator=g) * 0.02
    S = A @ A.transpose(1, 2) + torch.eye(3) * 1e-5
    cov = L(S[:, [0, 0, 0, 1, 1, 2], [0, 1, 2, 1, 2, 2]].contiguous())
    m2 = torch.zeros_like(means3D, requires_grad=True)
    E = torch.Tensor([])
    out = _RasterizeGaussians.apply(means3D, m2, E, cols, segs, opac, E, E, cov, st)
    fn = out[0].grad_fn
    ups = [torch.randn_like(out[k]) for k in (0, 2, 3, 4)]
    grads = fn.apply(ups[0], None, ups[1], ups[2], ups[3])  # the autograd node's backward
    # inputs: means3D, means2D, sh, colors, segments, opacities, scales, rotations, cov3D, settings
    assert grads[2] is None and grads[6] is None and grads[7] is None and grads[9] is None
    for i in (0, 1, 3, 4, 5, 8):
        assert grads[i] is not None and 0 not in grads[i].stride(), f"input {i}"
        grads[i].add_(0.0)  # writable in place


def test_backward_rejects_sh_after_colors_precomp_forward(gpu_available):
    """the C ABI's colour-source contract (include/gsr.h gsr_backward) is guarded.
    A backward given shs for a geom buffer whose forward took colors_precomp would read the SH
    direction Jacobian the forward never wrote; libgsr fails that call (RuntimeError through the
    binding) instead of returning garbage gradients with rc 0.  The matching call succeeds."""
    from diff_gaussian_rasterization import _C
    scene = synthetic_scene(3000, sh_degree=3, seed=72)
    cam = orbit_camera(1, 96, 64, 80.0)
    st = Hn.settings_for(cam, 3, "cuda")
    dev = "cuda"
    means3D, opac, segs = scene.means3D.to(dev), scene.opacities.to(dev), scene.segments.to(dev)
    scales, rots, shs = scene.scales.to(dev), scene.rotations.to(dev), scene.shs.to(dev)
    cols = torch.rand(scene.P, 3, device=dev)
    E = torch.Tensor([])
    fwd = _C.rasterize_gaussians(st.bg, means3D, cols, segs, opac, scales, rots, st.scale_modifier, E,
                                 st.viewmatrix, st.projmatrix, st.tanfovx, st.tanfovy, st.image_height,
                                 st.image_width, E, st.sh_degree, st.campos, st.prefiltered, st.debug)
    R, color, depth, segment, alpha, radii, geom, binning, img = fwd
    assert R > 0
    ups = (torch.randn_like(color), torch.randn_like(segment), torch.randn_like(depth), torch.randn_like(alpha))

    def backward(colors, sh):
        return _C.rasterize_gaussians_backward(st.bg, means3D, radii, colors, segs, scales, rots, st.scale_modifier,
                                               E, st.viewmatrix, st.projmatrix, st.tanfovx, st.tanfovy, *ups, sh,
                                               st.sh_degree, st.campos, geom, R, binning, img, alpha, st.debug)

    with pytest.raises(RuntimeError, match="colors_precomp"):
        backward(E, shs)
    g = backward(cols, E)
    torch.cuda.synchronize()
    assert torch.isfinite(g[3]).all() and float(g[1].abs().sum()) > 0


def test_multiview_backward_rejects_bad_view_before_any_launch(gpu_available):
    """the multi-view backward puts odd views' render backward on libgsr's auxiliary
    stream.  A view that fails its checks (here view 2 of 3: a geom buffer from a colors_precomp
    forward, backward given shs) must fail the call before anything is queued, so no auxiliary
    work can outlive the call unjoined.  The same three views with a consistent colour source
    then succeed."""
    from diff_gaussian_rasterization import _C
    scene = synthetic_scene(3000, sh_degree=3, seed=73)
    dev = "cuda"
    means3D, opac, segs = scene.means3D.to(dev), scene.opacities.to(dev), scene.segments.to(dev)
    scales, rots, shs = scene.scales.to(dev), scene.rotations.to(dev), scene.shs.to(dev)
    cols = torch.rand(scene.P, 3, device=dev)
    E = torch.Tensor([])
    views = []
    for v in range(3):
        cam = orbit_camera(v, 96, 64, 80.0)
        st = Hn.settings_for(cam, 3, dev)
        use_cols = v == 2
        R, color, depth, segment, alpha, radii, geom, binning, img = _C.rasterize_gaussians(
            st.bg, means3D, cols if use_cols else E, segs, opac, scales, rots, st.scale_modifier, E,
            st.viewmatrix, st.projmatrix, st.tanfovx, st.tanfovy, st.image_height, st.image_width,
            E if use_cols else shs, st.sh_degree, st.campos, st.prefiltered, st.debug)
        assert R > 0
        views.append(dict(bg=st.bg, viewmatrix=st.viewmatrix, projmatrix=st.projmatrix, tanfovx=st.tanfovx,
                          tanfovy=st.tanfovy, image_height=st.image_height, image_width=st.image_width,
                          campos=st.campos, radii=radii, geom=geom, binning=binning, img=img, num_rendered=R,
                          alpha=alpha, dL_dcolor=torch.randn_like(color), dL_dsegment=torch.randn_like(segment),
                          dL_ddepth=torch.randn_like(depth), dL_dalpha=torch.randn_like(alpha)))
    with pytest.raises(RuntimeError, match="colors_precomp"):
        _C.rasterize_gaussians_backward_multiview(views, means3D, E, segs, scales, rots, 1.0, E, shs, 3, False)
    torch.cuda.synchronize()
    out, d2 = _C.rasterize_gaussians_backward_multiview(views[:2], means3D, E, segs, scales, rots, 1.0, E, shs, 3,
                                                        False)
    torch.cuda.synchronize()
    assert torch.isfinite(out[3]).all() and float(out[5].abs().sum()) > 0
