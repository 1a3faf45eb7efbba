"""The C++ host binding (csrc/host_ext.cpp, module gsr_host) loads without a GPU and exports the
entry points the drop-in API calls: the single-view forward / backward, the autograd function and
its sink / stamp hooks.  (Its results: tests/test_gpu_host_ext.py, test_gpu_host_autograd.py.)"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3d_gaussian_magic_change-segment_3dgs_amd"))


def test_host_ext_exports():
    import torch  # noqa: F401  (the extension links against torch's libraries)
    from diff_gaussian_rasterization import _host
    mod = _host.load()
    if mod is None:
        pytest.skip("gsr_host not built from these sources (__graft_entry__.build())")
    for name in ("rasterize", "rasterize_gaussians", "rasterize_gaussians_backward", "set_sinks", "set_sink_backward",
                 "stamps", "version", "lib_ns"):
        assert callable(getattr(mod, name)), name
    assert mod.stamps(False) == []
    assert mod.version()


def test_rasterize_gaussians_dispatch(monkeypatch):
    """rasterize_gaussians() hands the C++ autograd route its arguments in RasterizeFn's order
    (settings fields by name), feeds the binning-capacity window with the count it returns, and
    keeps the Python function for debug mode and for forwards inside defer_sh_gradients."""
    import torch
    import diff_gaussian_rasterization as dgr
    from diff_gaussian_rasterization import _C
    calls, py_calls = [], []

    class Fake:
        def rasterize(self, *a):
            calls.append(a)
            return ("color", "radii", "depth", "alpha", "segment", 77)

        def set_sinks(self, n):
            calls.append(("sinks", n))

    monkeypatch.setattr(_C, "_HOST_AUTOGRAD", Fake())
    monkeypatch.setattr(_C, "_last_rendered", {})
    monkeypatch.setattr(dgr._RasterizeGaussians, "apply", lambda *a: py_calls.append(a) or "python route")
    st = dgr.GaussianRasterizationSettings(
        image_height=8, image_width=12, tanfovx=0.5, tanfovy=0.25, bg=torch.zeros(3), scale_modifier=1.5,
        viewmatrix=torch.eye(4), projmatrix=2 * torch.eye(4), sh_degree=2, campos=torch.ones(3), prefiltered=False,
        debug=False)
    m = torch.zeros(5, 3)
    args = (m, m, "sh", "col", "seg", "op", "sc", "rot", "cov")
    assert dgr.rasterize_gaussians(*args, st) == ("color", "radii", "depth", "alpha", "segment")
    a = calls[0]
    assert a[0] is m and a[1] is m and a[2:9] == args[2:]
    assert a[9] is st.bg and a[10] is st.viewmatrix and a[11] is st.projmatrix and a[12] is st.campos
    assert a[13:20] == (1.5, 0.5, 0.25, 8, 12, 2, False) and a[20] == 0  # no guess before the first count
    assert _C._last_rendered[m.device] == [77]
    dgr.rasterize_gaussians(*args, st)
    assert calls[-1][20] == 77 + 77 // 7 + 4096  # the window's guess
    assert dgr.rasterize_gaussians(*args, st._replace(debug=True)) == "python route"
    with dgr.defer_sh_gradients(object()):
        assert dgr.rasterize_gaussians(*args, st) == "python route"
    assert ("sinks", 1) in calls and calls[-1] == ("sinks", 0)
    assert len(py_calls) == 2
