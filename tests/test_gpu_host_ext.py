"""The C++ host binding (csrc/host_ext.cpp, module gsr_host) against the ctypes route of _C.py:
the same libgsr calls with the same buffers, so every output and gradient must be bit-identical,
on every argument path (SH / precomputed colours, scale+rotation / precomputed covariance,
absent segments, an upstream gradient autograd did not materialise, P = 0), with the same
errors.  It is the route the drop-in API takes when built (profiles/round6_*_host_overhead.txt
for its host time)."""
import pytest
import torch

import harness as Hn
from gsr_tools.scene import synthetic_scene, orbit_camera

pytestmark = pytest.mark.gpu


def _both(monkeypatch, fn):
    # the Python autograd function on both sides (tests/test_gpu_host_autograd.py: the C++ one)
    from diff_gaussian_rasterization import _C
    assert _C._HOST is not None, "gsr_host not built (__graft_entry__.build())"
    monkeypatch.setattr(_C, "_HOST_AUTOGRAD", None)
    a = fn()
    monkeypatch.setattr(_C, "_HOST", None)
    b = fn()
    monkeypatch.undo()
    return a, b


@pytest.mark.parametrize("variant", ["sh", "colors", "cov3D", "no_segments", "bg"])
def test_host_ext_matches_ctypes(gpu_available, monkeypatch, variant):
    scene = synthetic_scene(30000, sh_degree=3, seed=61)
    cam = orbit_camera(3, 320, 240, 300.0)
    grads = Hn.upstream_grads(cam.height, cam.width)
    kw = {}
    if variant == "colors":
        kw["colors_precomp"] = torch.rand(scene.P, 3, generator=torch.Generator().manual_seed(2))
    if variant == "cov3D":
        g = torch.Generator().manual_seed(3)
        A = torch.randn(scene.P, 3, 3, generator=g) * 0.01
        C = A @ A.transpose(1, 2) + torch.eye(3) * 1e-5
        kw["cov3D_precomp"] = C[:, [0, 0, 0, 1, 1, 2], [0, 1, 2, 1, 2, 2]].contiguous()
    if variant == "no_segments":
        kw["use_segments"] = False
    if variant == "bg":
        kw["bg"] = (0.2, 0.5, 0.9)
    a, b = _both(monkeypatch, lambda: Hn.run_gsr(scene, cam, grads=grads, **kw))
    assert a["num_rendered"] == b["num_rendered"] > 0
    for k in ("color", "depth", "alpha", "segment", "radii", "point_list", "n_contrib"):
        assert (a[k] == b[k]).all(), k
    for k in a["grads"]:
        assert (a["grads"][k] == b["grads"][k]).all(), k


def test_host_ext_unmaterialised_grads_and_errors(gpu_available, monkeypatch):
    from diff_gaussian_rasterization import _C, rasterize_gaussians
    scene = synthetic_scene(5000, sh_degree=1, seed=62)
    cam = orbit_camera(1, 160, 120, 150.0)
    st = Hn.settings_for(cam, 1, "cuda")
    leaf = lambda t: t.detach().cuda().clone().requires_grad_(True)
    E = torch.Tensor([])

    def run():
        d = {k: leaf(getattr(scene, k)) for k in ("means3D", "shs", "opacities", "scales", "rotations", "segments")}
        m2 = torch.zeros_like(d["means3D"], requires_grad=True)
        color, radii, depth, alpha, seg = rasterize_gaussians(d["means3D"], m2, d["shs"], E, d["segments"],
                                                              d["opacities"], d["scales"], d["rotations"], E, st)
        color.sum().backward()  # depth / alpha / segment gradients are not materialised (None)
        return [color.detach()] + [d[k].grad for k in d] + [m2.grad]

    a, b = _both(monkeypatch, run)
    for x, y in zip(a, b):
        assert torch.equal(x, y)
    assert _C._HOST is not None
    with pytest.raises(RuntimeError, match="means3D must have dimensions"):
        _C.rasterize_gaussians(st.bg, torch.zeros(4, 2, device="cuda"), E, E, E, E, E, 1.0, E, st.viewmatrix,
                               st.projmatrix, 1.0, 1.0, 8, 8, E, 0, st.campos, False, False)
    with pytest.raises(RuntimeError, match="must be a float32 tensor"):
        _C.rasterize_gaussians(st.bg, torch.zeros(4, 3, device="cuda", dtype=torch.float64), E, E, E, E, E, 1.0, E,
                               st.viewmatrix, st.projmatrix, 1.0, 1.0, 8, 8, E, 0, st.campos, False, False)
    out = _C.rasterize_gaussians(st.bg, torch.zeros(0, 3, device="cuda"), E, E, E, E, E, 1.0, E, st.viewmatrix,
                                 st.projmatrix, 1.0, 1.0, 8, 12, E, 0, st.campos, False, False)
    assert out[0] == 0 and out[1].shape == (3, 8, 12) and float(out[1].abs().sum()) == 0.0
