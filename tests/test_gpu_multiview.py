"""Multi-view backward (include/gsr.h gsr_backward_multiview): the parameter
gradients of a batch of views in one call must equal the sum of the single-view
drop-in gradients, and each view's dmeans2D must equal that view's own.

Tolerance: the sums over views are taken in a different order (per-view transforms
of summed terms vs sums of per-view results; dscales/drot from the summed dcov3D),
so parameter gradients agree to fp32 rounding: normwise |diff| <= 1e-5 * |ref| per
tensor.  dmeans2D runs the identical per-view code: bit-exact."""
import numpy as np
import pytest
import torch

import harness as Hn
from gsr_tools.scene import synthetic_scene, orbit_camera

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _leaves(scene, colors=False, cov=False, sh_take=None):
    L = lambda t: t.detach().to(DEV).clone().requires_grad_(True)
    d = {"means3D": L(scene.means3D), "opacities": L(scene.opacities), "segments": L(scene.segments)}
    if colors:
        d["colors_precomp"] = L(torch.rand(scene.P, 3, generator=torch.Generator().manual_seed(5)))
    else:
        shs = scene.shs if sh_take is None else scene.shs[:, :sh_take].contiguous()
        d["shs"] = L(shs)
    if cov:
        g = torch.Generator().manual_seed(6)
        A = torch.randn(scene.P, 3, 3, generator=g) * 0.01
        C = A @ A.transpose(1, 2) + torch.eye(3) * 1e-5
        d["cov3D_precomp"] = L(C[:, [0, 0, 0, 1, 1, 2], [0, 1, 2, 1, 2, 2]].contiguous())
    else:
        d["scales"], d["rotations"] = L(scene.scales), L(scene.rotations)
    return d


def _views(n, deg, W=160, H=120):
    cams = [orbit_camera(i, W, H, 150.0, n_views=max(n, 3)) for i in range(n)]
    return [(Hn.settings_for(c, deg, DEV), Hn.upstream_grads(H, W, seed=10 + i)) for i, c in enumerate(cams)]


def _kw(d):
    E = torch.Tensor([])
    return dict(sh=d.get("shs", E), colors_precomp=d.get("colors_precomp", E), segments=d["segments"],
                opacities=d["opacities"], scales=d.get("scales", E), rotations=d.get("rotations", E),
                cov3Ds_precomp=d.get("cov3D_precomp", E))


def _single(d, views):
    from diff_gaussian_rasterization import rasterize_gaussians
    total, d2 = {}, []
    for st, ups in views:
        m2 = torch.zeros_like(d["means3D"], requires_grad=True)
        color, radii, depth, alpha, seg = rasterize_gaussians(d["means3D"], m2, raster_settings=st, **_kw(d))
        grads = torch.autograd.grad([color, depth, alpha, seg], [d[k] for k in d] + [m2],
                                    [ups["color"].to(DEV), ups["depth"].to(DEV), ups["alpha"].to(DEV),
                                     ups["segment"].to(DEV)], allow_unused=True)
        for k, gr in zip(d, grads[:-1]):
            if gr is not None:
                total[k] = total.get(k, 0) + gr.double()
        d2.append(grads[-1])
    return total, d2


def _multi(d, views):
    from diff_gaussian_rasterization import rasterize_gaussians_multiview
    m2s = [torch.zeros_like(d["means3D"], requires_grad=True) for _ in views]
    outs = rasterize_gaussians_multiview(d["means3D"], m2s, raster_settings_list=[v[0] for v in views], **_kw(d))
    tensors, gouts = [], []
    for (color, radii, depth, alpha, seg), (_, ups) in zip(outs, views):
        tensors += [color, depth, alpha, seg]
        gouts += [ups["color"].to(DEV), ups["depth"].to(DEV), ups["alpha"].to(DEV), ups["segment"].to(DEV)]
    grads = torch.autograd.grad(tensors, [d[k] for k in d] + m2s, gouts, allow_unused=True)
    n = len(d)
    return dict(zip(d, grads[:n])), list(grads[n:]), outs


def _check(d, views):
    ref, ref_d2 = _single(d, views)
    got, got_d2, outs = _multi(d, views)
    for k, r in ref.items():
        g = got[k].double()
        err = float((g - r).norm() / max(float(r.norm()), 1e-30))
        assert err <= 1e-5, f"{k}: normwise error {err:.2e}"
    for v, (a, b) in enumerate(zip(got_d2, ref_d2)):
        assert torch.equal(a, b), f"view {v}: dmeans2D differs (max {float((a - b).abs().max()):.3e})"
    return outs


@pytest.mark.parametrize("n_views", [1, 3, 8])
def test_multiview_equals_sum_of_views_sh3(gpu_available, n_views):
    scene = synthetic_scene(6000, sh_degree=3, seed=41)
    _check(_leaves(scene), _views(n_views, 3))


def test_multiview_forward_outputs_equal_single(gpu_available):
    from diff_gaussian_rasterization import rasterize_gaussians
    scene = synthetic_scene(3000, sh_degree=3, seed=42)
    d = _leaves(scene)
    views = _views(2, 3)
    outs = _check(d, views)
    for (st, _), o in zip(views, outs):
        r = rasterize_gaussians(d["means3D"], torch.zeros_like(d["means3D"]), raster_settings=st, **_kw(d))
        for a, b in zip(o, r):
            assert torch.equal(a, b)


@pytest.mark.parametrize("variant", ["colors_cov", "sh_deg1_m16", "sh_m9_unstaged"])
def test_multiview_argument_paths(gpu_available, variant):
    if variant == "colors_cov":
        scene = synthetic_scene(4000, sh_degree=3, seed=43)
        d, views = _leaves(scene, colors=True, cov=True), _views(3, 3)
    elif variant == "sh_deg1_m16":
        scene = synthetic_scene(4000, sh_degree=3, seed=44)
        d, views = _leaves(scene), _views(3, 1)
    else:
        scene = synthetic_scene(4000, sh_degree=2, seed=45)  # M = 9: rows of 27 floats, per-thread path
        d, views = _leaves(scene), _views(3, 2)
    _check(d, views)


def test_multiview_view_with_nothing_visible(gpu_available):
    scene = synthetic_scene(2000, sh_degree=3, seed=46)
    d = _leaves(scene)
    views = _views(2, 3)
    import copy
    far = orbit_camera(0, 160, 120, 150.0, radius=-4.0)  # camera behind the scene, looking away
    views.append((Hn.settings_for(far, 3, DEV), Hn.upstream_grads(120, 160, seed=99)))
    _check(d, views)


# ---- deferred SH gradients (include/gsr.h gsr_backward_multiview_deferred_sh +
# gsr_sh_backward): the split into "rows now, SH later" runs the same per-Gaussian
# arithmetic in the same order, so the completed gradients are bit-identical.
class _Sink:
    def __init__(self):
        self.entries = []

    def sh_rows(self, B, P, device):
        from diff_gaussian_rasterization import _C
        return torch.full((B * _C.sh_rows_floats(P),), float("nan"), dtype=torch.float32, device=device)

    def record(self, rows, B, means3D, sh, degree, dsh, dmeans3D, inputs=()):
        self.entries.append((rows, B, means3D, sh, degree, dsh, dmeans3D))


@pytest.mark.parametrize("n_views,deg,sh_take", [(1, 3, None), (3, 3, None), (3, 2, 9)])
def test_deferred_sh_completes_to_multiview(gpu_available, n_views, deg, sh_take):
    from diff_gaussian_rasterization import _C, defer_sh_gradients
    scene = synthetic_scene(5000, sh_degree=3, seed=47)
    d = _leaves(scene, sh_take=sh_take)
    views = _views(n_views, deg)
    ref, ref_d2, _ = _multi(d, views)
    sink = _Sink()
    with defer_sh_gradients(sink):
        got, got_d2, _ = _multi(d, views)
    assert len(sink.entries) == 1
    rows, B, means3D, sh, degree, dsh, dmeans3D = sink.entries[0]
    assert B == n_views and dsh.data_ptr() == got["shs"].data_ptr()
    P = scene.P
    ch = _C.sh_rows_floats(P)
    for v, (st, _) in enumerate(views):  # each view's camera centre travels with its rows
        assert torch.equal(rows[v * ch + ch - 64:v * ch + ch - 61], st.campos.float())
    _C.sh_backward(rows, B, means3D.detach(), sh.detach(), degree, dsh, dmeans3D)
    for k in ref:
        assert torch.equal(got[k], ref[k]), f"{k} differs after the SH completion"
    for a, b in zip(got_d2, ref_d2):
        assert torch.equal(a, b)


def test_sh_backward_two_batches_sum(gpu_available):
    """Rows of two batches completed together equal the multi-view backward of all
    views (what every rank computes after the all-gather)."""
    from diff_gaussian_rasterization import _C, defer_sh_gradients
    scene = synthetic_scene(4000, sh_degree=3, seed=48)
    d = _leaves(scene)
    views = _views(4, 3)
    ref, _, _ = _multi(d, views)
    parts = []
    for half in (views[:2], views[2:]):
        sink = _Sink()
        with defer_sh_gradients(sink):
            g, _, _ = _multi(d, half)
        parts.append((g, sink.entries[0]))
    (g0, e0), (g1, e1) = parts
    rows_all = torch.cat([e0[0], e1[0]])
    # the non-SH blocks are summed as an all-reduce would; then the SH completion
    dm = (g0["means3D"] + g1["means3D"]).contiguous()
    dsh = torch.empty_like(g0["shs"])
    _C.sh_backward(rows_all, 4, d["means3D"].detach(), d["shs"].detach(), 3, dsh, dm)
    for k, got in (("shs", dsh), ("means3D", dm), ("opacities", g0["opacities"] + g1["opacities"]),
                   ("scales", g0["scales"] + g1["scales"]), ("rotations", g0["rotations"] + g1["rotations"])):
        r = ref[k].double()
        err = float((got.double() - r).norm() / max(float(r.norm()), 1e-30))
        assert err <= 1e-6, f"{k}: normwise error {err:.2e}"


def test_sh_exchange_single_rank_equals_dropin(gpu_available):
    """gsr_tools.dp.ShExchange around the drop-in single-view backward (world size 1
    over gloo): the exchanged bucket equals the drop-in backward's bucket."""
    import os
    import socket
    import torch.distributed as dist
    from diff_gaussian_rasterization import defer_sh_gradients
    from gsr_tools import dp
    scene = synthetic_scene(5000, sh_degree=3, seed=49)
    d = _leaves(scene)
    views = _views(1, 3)
    ref, _ = _single(d, views)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        from diff_gaussian_rasterization import rasterize_gaussians
        st, ups = views[0]
        m2 = torch.zeros_like(d["means3D"], requires_grad=True)
        color, radii, depth, alpha, seg = rasterize_gaussians(d["means3D"], m2, raster_settings=st, **_kw(d))
        ex = dp.ShExchange()
        with defer_sh_gradients(ex):
            grads = torch.autograd.grad([color, depth, alpha, seg], [d[k] for k in d],
                                        [ups["color"].to(DEV), ups["depth"].to(DEV), ups["alpha"].to(DEV),
                                         ups["segment"].to(DEV)])
        assert len(ex.entries) == 1
        ex.start().wait()  # nothing reads the deferred gradients before this
        got = {k: g.double() for k, g in zip(d, grads)}
    finally:
        dist.destroy_process_group()
    for k, r in ref.items():
        err = float((got[k] - r).norm() / max(float(r.norm()), 1e-30))
        assert err <= 1e-6, f"{k}: normwise error {err:.2e}"


def test_deferred_sh_single_view_completes_to_dropin(gpu_available):
    """gsr_backward_deferred_sh (one view per rank: the single-view backward writing its
    exchange rows instead of dsh) completed by sh_backward gives the drop-in single-view
    gradients bit for bit: dmeans3D carries the direction term already, dsh is rebuilt from
    the row with the same basis products."""
    from diff_gaussian_rasterization import _C, defer_sh_gradients, rasterize_gaussians
    scene = synthetic_scene(5000, sh_degree=3, seed=50)
    d = _leaves(scene)
    (st, ups), = _views(1, 3)

    def run():
        m2 = torch.zeros_like(d["means3D"], requires_grad=True)
        color, radii, depth, alpha, seg = rasterize_gaussians(d["means3D"], m2, raster_settings=st, **_kw(d))
        return torch.autograd.grad([color, depth, alpha, seg], [d[k] for k in d] + [m2],
                                   [ups["color"].to(DEV), ups["depth"].to(DEV), ups["alpha"].to(DEV),
                                    ups["segment"].to(DEV)])

    ref = run()
    sink = _Sink()
    with defer_sh_gradients(sink):
        got = run()
    assert len(sink.entries) == 1
    rows, B, means3D, sh, degree, dsh, dmeans3D = sink.entries[0]
    assert B == 1 and dsh.data_ptr() == got[list(d).index("shs")].data_ptr()
    ch = _C.sh_rows_floats(scene.P)
    assert torch.equal(rows[ch - 64:ch - 61], st.campos.float())
    _C.sh_backward(rows, 1, means3D.detach(), sh.detach(), degree, dsh, dmeans3D)
    for k, a, b in zip(list(d) + ["means2D"], got, ref):
        assert torch.equal(a, b), f"{k} differs after the SH completion"


def test_multiview_deferred_forward_rebinning(gpu_available):
    """The multi-view forward launches every view before waiting for any num_rendered
    (gsr_forward_deferred / gsr_forward_wait).  With a binning guess far below the views'
    counts, every view takes gsr_forward_wait's GSR_NEED_BINNING path and re-runs stage B with
    the exact buffer: outputs still equal the single-view drop-in's, bit for bit."""
    from diff_gaussian_rasterization import _C, rasterize_gaussians
    scene = synthetic_scene(20000, sh_degree=3, seed=47)
    d = _leaves(scene)
    views = _views(3, 3, W=320, H=240)
    ref = [rasterize_gaussians(d["means3D"], torch.zeros_like(d["means3D"]), raster_settings=st, **_kw(d))
           for st, _ in views]
    assert all(int((r[1] > 0).sum()) > 0 for r in ref)
    dev = d["means3D"].device
    _C._last_rendered[dev] = [1]  # guess: 1 + 4096 instances, far below the counts
    got, _, outs = _multi(d, views)
    for o, r in zip(outs, ref):
        for a, b in zip(o, r):
            assert torch.equal(a, b)
    assert max(_C._last_rendered[dev]) > 4097  # the counts were above the guess


@pytest.mark.parametrize("streams", [3, 4])
def test_multiview_forward_streams(gpu_available, streams, monkeypatch):
    """Views dealt over more forward streams (GSR_MV_FWD_STREAMS): the same outputs and gradients."""
    import diff_gaussian_rasterization as dgr
    monkeypatch.setattr(dgr, "_MV_FWD_STREAMS", streams)
    scene = synthetic_scene(4000, sh_degree=3, seed=48)
    d = _leaves(scene)
    _check(d, _views(5, 3))


def test_multiview_forward_end_failure_frees_tickets(gpu_available, monkeypatch):
    """an error while ending view v of a multi-view forward (e.g. an out-of-memory
    stage-B buffer after gsr_forward_wait) must still end views v+1.. (their deferred tickets
    are per-thread pinned slots, 16 of them) and join the side streams.  Ten failed batches of
    four views would leak 20 tickets without that; a batch after them must still work."""
    from diff_gaussian_rasterization import _C
    import diff_gaussian_rasterization as dgr
    scene = synthetic_scene(6000, sh_degree=3, seed=49)
    d = _leaves(scene)
    views = _views(4, 3)
    real_end = _C.rasterize_gaussians_end
    calls = {"n": 0}

    def failing_end(h):
        out = real_end(h)
        calls["n"] += 1
        if calls["n"] % 4 == 2:
            raise RuntimeError("injected failure after the wait")
        return out

    _multi(d, views)  # warm the binning guess so that begin() defers
    monkeypatch.setattr(_C, "rasterize_gaussians_end", failing_end)
    for _ in range(10):
        calls["n"] = 0
        with pytest.raises(RuntimeError, match="injected"):
            dgr.rasterize_gaussians_multiview(d["means3D"], [torch.zeros_like(d["means3D"]) for _ in views],
                                              raster_settings_list=[st for st, _ in views], **_kw(d))
    monkeypatch.setattr(_C, "rasterize_gaussians_end", real_end)
    torch.cuda.synchronize()
    _check(d, views)
