"""C-ABI checks that need no GPU: libgsr.so loads, exports every symbol that
include/gsr.h declares, size queries behave, errors are reported through
gsr_last_error, and the Python layer rejects bad arguments before any launch."""
import ctypes
import os
import re

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "gsr.h")


def declared_symbols():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"GSR_API\s+[\w\s\*]*?\b(gsr_\w+)\s*\(", txt)))


def test_header_declares_the_boundary():
    syms = declared_symbols()
    for s in ("gsr_forward_geometry", "gsr_forward_render", "gsr_backward", "gsr_mark_visible", "gsr_last_error",
              "gsr_geom_bytes", "gsr_binning_bytes", "gsr_img_bytes", "gsr_backward_scratch_bytes"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    from diff_gaussian_rasterization import _C
    lib = ctypes.CDLL(_C.LIB_PATH)
    for s in declared_symbols():
        assert hasattr(lib, s), f"{s} declared in include/gsr.h but not exported"
    assert sorted(_C.EXPORTED_SYMBOLS) == declared_symbols()
    assert _C.version().startswith("gsr")


def test_size_queries():
    from diff_gaussian_rasterization import _C
    L = _C._lib
    assert L.gsr_geom_bytes(1_000_000) > 64 * 1_000_000
    assert L.gsr_geom_bytes(2000) > L.gsr_geom_bytes(1000) > L.gsr_geom_bytes(0)
    assert L.gsr_binning_bytes(10_000_000) >= 24 * 10_000_000
    assert L.gsr_img_bytes(1920, 1080) >= 120 * 68 * (8 + 256 * 4)
    assert L.gsr_backward_scratch_bytes(100) >= 100 * 48


def test_errors_reported_without_touching_the_device():
    from diff_gaussian_rasterization import _C
    L = _C._lib
    s = _C._Settings()
    s.P, s.W, s.H = 10, 64, 64
    inp = _C._Inputs()  # means3D NULL
    nr = ctypes.c_int(-1)
    rc = L.gsr_forward_geometry(ctypes.byref(s), ctypes.byref(inp), None, None, None, ctypes.byref(nr))
    assert rc != 0 and b"means3D" in L.gsr_last_error()
    inp.means3D = inp.opacities = 16
    inp.shs, inp.colors_precomp = 16, 32
    rc = L.gsr_forward_geometry(ctypes.byref(s), ctypes.byref(inp), None, None, None, ctypes.byref(nr))
    assert rc != 0 and b"SHs or precomputed colors" in L.gsr_last_error()
    inp.colors_precomp = None
    s.D, s.M = 3, 9
    inp.scales, inp.rotations = 16, 32
    rc = L.gsr_forward_geometry(ctypes.byref(s), ctypes.byref(inp), None, None, None, ctypes.byref(nr))
    assert rc != 0 and b"SH degree" in L.gsr_last_error()
    assert L.gsr_debug_copy(b"no_such_field", 1, 16, 16, 0, None, None, None, 16, None) == -1


def test_python_api_rejects_cpu_tensors():
    """The product path has no CPU fallback: CPU inputs fail loudly."""
    from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer
    st = GaussianRasterizationSettings(16, 16, 0.5, 0.5, torch.zeros(3), 1.0, torch.eye(4), torch.eye(4), 0,
                                       torch.zeros(3), False, False)
    m = torch.zeros(4, 3)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        GaussianRasterizer(st)(means3D=m, means2D=m, opacities=torch.ones(4, 1), shs=torch.ones(4, 1, 3),
                               scales=m, rotations=torch.ones(4, 4))
    with pytest.raises(Exception, match="excatly one of either SHs"):
        GaussianRasterizer(st)(means3D=m, means2D=m, opacities=torch.ones(4, 1), scales=m,
                               rotations=torch.ones(4, 4))


def test_grad_arena_layout_bucket_first():
    from diff_gaussian_rasterization import _C
    lay = _C.grad_arena_layout(10, 16)
    assert lay["bucket"] == (0, 10 * (3 + 48 + 1 + 3 + 4 + 2))
    assert lay["dmeans3D"][0] == 0 and lay["dsegments"][0] + 20 == lay["bucket"][1]
