"""The drop-in rasterize_gaussians' C++ autograd route (csrc/host_ext.cpp RasterizeFn) against
the Python _RasterizeGaussians over the same binding and against the ctypes route: the same
libgsr calls with the same buffers, so every output and gradient must be bit-identical on every
argument path (SH / precomputed colours, scale+rotation / precomputed covariance, absent
segments), for any subset of inputs that need a gradient and of outputs that get one, with
retain_graph, under no_grad, at P = 0, with the same errors, and with a defer_sh_gradients sink
entered between the forward and the backward.  Debug mode keeps the Python function (snapshot
dumps).  profiles/round6_*_host_overhead.txt: the host time each route costs."""
import pytest
import torch

import harness as Hn
from gsr_tools.scene import orbit_camera, synthetic_scene

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _route(monkeypatch, route):
    from diff_gaussian_rasterization import _C
    monkeypatch.undo()
    assert _C._HOST_AUTOGRAD is not None, "gsr_host not built (__graft_entry__.build())"
    if route in ("py", "ctypes"):
        monkeypatch.setattr(_C, "_HOST_AUTOGRAD", None)
    if route == "ctypes":
        monkeypatch.setattr(_C, "_HOST", None)


def _inputs(scene, variant="sh", needs=None):
    def L(name, t):
        return t.detach().to(DEV).clone().requires_grad_(needs is None or name in needs)
    E = torch.Tensor([])
    d = dict(means3D=L("means3D", scene.means3D), sh=L("sh", scene.shs), colors_precomp=E,
             segments=L("segments", scene.segments), opacities=L("opacities", scene.opacities),
             scales=L("scales", scene.scales), rotations=L("rotations", scene.rotations), cov3Ds_precomp=E)
    if variant == "colors":
        d["sh"] = E
        d["colors_precomp"] = L("colors_precomp", torch.rand(scene.P, 3, generator=torch.Generator().manual_seed(2)))
    if variant == "cov3D":
        g = torch.Generator().manual_seed(3)
        A = torch.randn(scene.P, 3, 3, generator=g) * 0.01
        C = A @ A.transpose(1, 2) + torch.eye(3) * 1e-5
        d["scales"] = d["rotations"] = E
        d["cov3Ds_precomp"] = L("cov3Ds_precomp", C[:, [0, 0, 0, 1, 1, 2], [0, 1, 2, 1, 2, 2]].contiguous())
    if variant == "no_segments":
        d["segments"] = E
    return d


def _forward(d, st, m2_grad=True):
    from diff_gaussian_rasterization import rasterize_gaussians
    m2 = torch.zeros_like(d["means3D"], requires_grad=m2_grad)
    out = rasterize_gaussians(d["means3D"], m2, d["sh"], d["colors_precomp"], d["segments"], d["opacities"],
                              d["scales"], d["rotations"], d["cov3Ds_precomp"], st)
    assert isinstance(out, tuple) and len(out) == 5
    return dict(zip(("color", "radii", "depth", "alpha", "segment"), out)), m2


def _grads(d, m2):
    g = {k: t.grad for k, t in d.items() if t.numel() > 0}
    g["means2D"] = m2.grad
    return {k: None if v is None else v.clone() for k, v in g.items()}


def _assert_same(a, b):
    assert a.keys() == b.keys()
    for k in a:
        if a[k] is None or b[k] is None:
            assert a[k] is None and b[k] is None, k
        else:
            assert torch.equal(a[k], b[k]), k


def _scene_cam():
    return synthetic_scene(30000, sh_degree=3, seed=71), orbit_camera(2, 320, 240, 300.0)


@pytest.mark.parametrize("variant", ["sh", "colors", "cov3D", "no_segments", "bg"])
def test_cpp_autograd_matches_python_function(gpu_available, monkeypatch, variant):
    from diff_gaussian_rasterization import _C
    scene, cam = _scene_cam()
    st = Hn.settings_for(cam, 3, DEV, bg=(0.2, 0.5, 0.9) if variant == "bg" else (0.0, 0.0, 0.0))
    ups = Hn.upstream_grads(cam.height, cam.width)
    res = {}
    for route in ("cpp", "py", "ctypes"):
        _route(monkeypatch, route)
        d = _inputs(scene, variant)
        out, m2 = _forward(d, st)
        node = out["color"].grad_fn.name()
        assert ("RasterizeFn" in node) == (route == "cpp"), (route, node)
        assert not out["radii"].requires_grad
        if route == "cpp":
            assert _C._last_rendered[d["means3D"].device][-1] > 0  # the capacity guess is fed
        names = ("color", "depth", "alpha", "segment")
        torch.autograd.backward([out[k] for k in names], [ups[k].to(DEV) for k in names])
        res[route] = ({k: v.detach().clone() for k, v in out.items()}, _grads(d, m2))
    monkeypatch.undo()
    for route in ("py", "ctypes"):
        _assert_same(res["cpp"][0], res[route][0])
        _assert_same(res["cpp"][1], res[route][1])


def test_cpp_autograd_partial_needs_retain_and_no_grad(gpu_available, monkeypatch):
    """Only some inputs need a gradient (the others get none, as _finish_grads hands back), only
    the colour output gets one (the rest are not materialised), a second backward over the
    retained graph accumulates the same gradients, and a no_grad forward builds no graph."""
    scene, cam = _scene_cam()
    st = Hn.settings_for(cam, 3, DEV)
    ups = Hn.upstream_grads(cam.height, cam.width)
    res = {}
    for route in ("cpp", "py"):
        _route(monkeypatch, route)
        d = _inputs(scene, needs=("means3D", "opacities", "rotations"))
        out, m2 = _forward(d, st, m2_grad=False)
        out["color"].backward(ups["color"].to(DEV), retain_graph=True)
        once = _grads(d, m2)
        out["color"].backward(ups["color"].to(DEV))
        twice = _grads(d, m2)
        with torch.no_grad():
            ng, _ = _forward(_inputs(scene), st)
        assert ng["color"].grad_fn is None and not ng["color"].requires_grad
        for k in ("color", "depth", "alpha", "segment", "radii"):
            assert torch.equal(ng[k], out[k].detach()), k
        res[route] = (once, twice)
    monkeypatch.undo()
    for a, b in zip(res["cpp"], res["py"]):
        _assert_same(a, b)
    once, twice = res["cpp"]
    for k in ("means3D", "opacities", "rotations"):
        assert once[k] is not None and torch.equal(twice[k], once[k] + once[k]), k
    for k in ("sh", "segments", "scales", "means2D"):
        assert once[k] is None, k


def test_cpp_autograd_sink_entered_after_forward(gpu_available, monkeypatch):
    """A defer_sh_gradients sink entered between the forward and the backward: the C++ route's
    backward hands over to the sink's route (_cpp_sink_backward), as the Python function's does."""
    from diff_gaussian_rasterization import _C, defer_sh_gradients

    class Sink:
        def __init__(self):
            self.entries = []

        def sh_rows(self, B, P, device):
            return torch.full((B * _C.sh_rows_floats(P),), float("nan"), dtype=torch.float32, device=device)

        def record(self, rows, B, means3D, sh, degree, dsh, dmeans3D, inputs=()):
            self.entries.append((rows, B, means3D, sh, degree, dsh, dmeans3D))

    scene = synthetic_scene(5000, sh_degree=3, seed=72)
    cam = orbit_camera(1, 160, 120, 150.0)
    st = Hn.settings_for(cam, 3, DEV)
    ups = Hn.upstream_grads(cam.height, cam.width)
    names = ("color", "depth", "alpha", "segment")
    res = {}
    for route in ("cpp", "py"):
        _route(monkeypatch, route)
        d = _inputs(scene)
        out, m2 = _forward(d, st)
        sink = Sink()
        keys = [k for k in d if d[k].numel() > 0]
        with defer_sh_gradients(sink):
            got = torch.autograd.grad([out[k] for k in names], [d[k] for k in keys] + [m2],
                                      [ups[k].to(DEV) for k in names])
        assert len(sink.entries) == 1
        rows, B, means3D, sh, degree, dsh, dmeans3D = sink.entries[0]
        assert B == 1 and dsh.data_ptr() == got[keys.index("sh")].data_ptr()
        _C.sh_backward(rows, 1, means3D.detach(), sh.detach(), degree, dsh, dmeans3D)
        res[route] = dict(zip(keys + ["means2D"], (g.clone() for g in got)))
    monkeypatch.undo()
    _assert_same(res["cpp"], res["py"])


def test_cpp_autograd_errors_empty_and_debug(gpu_available, monkeypatch):
    from diff_gaussian_rasterization import GaussianRasterizer, rasterize_gaussians
    _route(monkeypatch, "cpp")
    cam = orbit_camera(1, 96, 64, 80.0)
    st = Hn.settings_for(cam, 0, DEV)
    E = torch.Tensor([])
    with pytest.raises(RuntimeError, match="means3D must have dimensions"):
        rasterize_gaussians(torch.zeros(4, 2, device=DEV), torch.zeros(4, 2, device=DEV), E, E, E, E, E, E, E, st)
    with pytest.raises(RuntimeError, match="must be a float32 tensor"):
        z = torch.zeros(4, 3, device=DEV, dtype=torch.float64)
        rasterize_gaussians(z, z, E, E, E, E, E, E, E, st)
    z = torch.zeros(0, 3, device=DEV, requires_grad=True)
    color, radii, depth, alpha, seg = rasterize_gaussians(z, torch.zeros(0, 3, device=DEV), E,
                                                          torch.zeros(0, 3, device=DEV), E,
                                                          torch.zeros(0, 1, device=DEV), E, E,
                                                          torch.zeros(0, 6, device=DEV), st)
    assert color.shape == (3, 64, 96) and float(color.abs().sum()) == 0.0 and radii.numel() == 0
    color.sum().backward()
    assert z.grad.shape == (0, 3)
    # debug mode: the Python function (it writes the snapshot dumps on a failure)
    scene = synthetic_scene(500, sh_degree=0, seed=73)
    d = _inputs(scene)
    out = GaussianRasterizer(st._replace(debug=True))(d["means3D"], torch.zeros_like(d["means3D"]), d["opacities"],
                                                      shs=d["sh"], segments=d["segments"], scales=d["scales"],
                                                      rotations=d["rotations"])
    assert "RasterizeFn" not in out[0].grad_fn.name()


def test_cpp_autograd_settings_changed_in_place(gpu_available, monkeypatch):
    """The settings' tensors are referenced, not version-checked, as the Python function keeps them
    (ctx.raster_settings): a camera moved in place between the forward and the backward gives both
    routes the same gradients and no error."""
    scene = synthetic_scene(5000, sh_degree=3, seed=74)
    cam = orbit_camera(1, 160, 120, 150.0)
    ups = Hn.upstream_grads(cam.height, cam.width)
    res = {}
    for route in ("cpp", "py"):
        _route(monkeypatch, route)
        st = Hn.settings_for(cam, 3, DEV)
        d = _inputs(scene)
        out, m2 = _forward(d, st)
        st.viewmatrix.mul_(1.0001)  # in place, after the forward
        st.campos.add_(0.001)
        out["color"].backward(ups["color"].to(DEV))
        res[route] = _grads(d, m2)
    monkeypatch.undo()
    _assert_same(res["cpp"], res["py"])
