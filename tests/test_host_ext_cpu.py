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
