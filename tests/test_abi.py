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
TRAIN_HEADER = os.path.join(ROOT, "include", "gsr_train.h")


def declared_symbols(header=HEADER):
    txt = open(header).read()
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


def test_library_exports_every_training_symbol():
    """include/gsr_train.h (SURVEY.md s8f kernels) is exported by the same library."""
    from diff_gaussian_rasterization import _C
    from gsr_train import _C as T
    lib = ctypes.CDLL(_C.LIB_PATH)
    syms = declared_symbols(TRAIN_HEADER)
    assert "gsr_adam_step" in syms and "gsr_activate" in syms
    for s in syms:
        assert hasattr(lib, s), f"{s} declared in include/gsr_train.h but not exported"
    assert sorted(T.EXPORTED_SYMBOLS) == syms


def test_training_calls_validate_without_the_device():
    from gsr_train import _C as T
    L = T._lib
    h = T.AdamHyper()
    assert L.gsr_adam_step(10, 16, 2, None, None, None, None, None, ctypes.byref(h), None) != 0
    assert b"null buffer" in L.gsr_last_error()
    assert L.gsr_adam_step(10, 17, 2, 16, 16, 16, 16, None, ctypes.byref(h), None) != 0
    assert b"invalid" in L.gsr_last_error()
    assert L.gsr_adam_step(0, 16, 2, None, None, None, None, None, ctypes.byref(h), None) == 0  # empty: no-op
    assert L.gsr_densify_stats(5, None, None, 16, None, 16, 16, None) != 0


def test_arena_spec_views_cover_reference_shapes():
    from gsr_train import ArenaSpec
    s = ArenaSpec(1001, 16)
    a = torch.arange(s.total, dtype=torch.float32)
    assert s.group(a, "f_dc").shape == (1001, 1, 3) and s.group(a, "f_rest").shape == (1001, 15, 3)
    assert s.group(a, "rotation").shape == (1001, 4) and s.group(a, "segment").shape == (1001, 2)
    assert float(s.group(a, "f_dc")[1, 0, 0]) == s.off[1] + 48  # [P,M,3] row-major, coefficient 0 first
    touched = torch.zeros(s.total, dtype=torch.int32)
    for n in ("xyz", "features", "opacity", "scaling", "rotation", "segment"):
        touched[s.off[("xyz", "features", "opacity", "scaling", "rotation", "segment").index(n)]:][
            :s.width[n] * s.P] += 1
    assert int(touched.max()) == 1  # blocks are disjoint


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
    assert L.gsr_debug_copy(b"no_such_field", 1, 16, 16, 0, 0, None, None, None, 16, None) == -1
    assert b"unknown field" in L.gsr_last_error()


def test_debug_copy_size_query():
    """gsr_debug_copy with dst = NULL returns the bytes a copy would take (no device access):
    the parity tests size their copies with it, so the host never assumes the library's layout."""
    from diff_gaussian_rasterization import _C
    L = _C._lib
    q = lambda name, P=7, W=100, H=40, I=33: L.gsr_debug_copy(name.encode(), P, W, H, I, 0,  # noqa: E731
                                                              None, None, None, None, None)
    T = 7 * 3
    assert q("rec") == 7 * 64 and q("point_list") == 33 * 4 and q("ranges") == T * 8
    assert q("n_contrib_tiles") == T * 256 * 4 and q("written") == 33
    sched = q("tile_order")
    assert sched % 4 == 0 and sched // 4 >= 2 * T + 4 + 64 + 64 * T  # order, sched words, counts, lists
    assert q("no_such_field") == -1
    # a field whose buffer is not passed copies nothing
    assert L.gsr_debug_copy(b"rec", 7, 100, 40, 33, 0, None, None, None, 16, None) == 0


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
    """The all-reduce bucket leads the gradient arena and matches the training
    arena of include/gsr_train.h block for block (64-float aligned blocks)."""
    import ctypes
    from diff_gaussian_rasterization import _C
    for P, M in ((10, 16), (1, 1), (1000, 9), (4097, 16)):
        lay = _C.grad_arena_layout(P, M)
        off = (ctypes.c_longlong * 7)()
        total = _C._lib.gsr_arena_layout(P, M, 2, off)
        names = ("dmeans3D", "dsh", "dopacity", "dscales", "drot", "dsegments")
        assert [lay[n][0] for n in names] == list(off)[:6]
        assert lay["bucket"] == (0, total) and total == off[6]
        assert all(o % 64 == 0 for o in off)
        for a, b in zip(names, names[1:]):  # blocks do not overlap
            assert lay[a][0] + lay[a][1] * P <= lay[b][0]
        assert lay["dsegments"][0] + 2 * P <= total < lay["dsegments"][0] + 2 * P + 64
        assert lay["dmeans2D"][0] == total and lay["total"][1] >= lay["dcov3D"][0] + 6 * P


def test_binning_capacity_inverts_the_size_query():
    """gsr_binning_capacity(bytes) is the largest C with gsr_binning_bytes(C) <= bytes: the
    layout capacity every call derives from a binning buffer's size (gsr.h)."""
    from diff_gaussian_rasterization import _C
    L = _C._lib
    assert L.gsr_binning_capacity(0) == -1
    for I in (0, 1, 63, 64, 4095, 4096, 100_000, 8_015_689, 9_218_042):
        b = L.gsr_binning_bytes(I)
        C = L.gsr_binning_capacity(b)
        assert C >= I and L.gsr_binning_bytes(C) == b and L.gsr_binning_bytes(C + 1) > b
        assert L.gsr_binning_capacity(b - 1) < I or I == 0
    t = torch.empty(L.gsr_binning_bytes(5000), dtype=torch.uint8)
    assert _C.binning_capacity(t) >= 5000 and _C.binning_capacity(torch.empty(0, dtype=torch.uint8)) == 0


def test_native_exchange_reports_errors_before_init():
    """The native exchange (csrc/dp.hip, include/gsr.h gsr_dp_*) fails loudly through
    gsr_last_error when it is used before gsr_dp_init or with bad arguments; none of these
    paths loads librccl or touches the device."""
    from diff_gaussian_rasterization import _C
    L = _C._lib
    assert L.gsr_dp_world() == 0
    assert L.gsr_dp_unique_id_bytes() == 128  # sizeof(ncclUniqueId)
    assert L.gsr_dp_finalize() == 0  # finalize without init is a no-op
    assert L.gsr_dp_get_unique_id(None) != 0 and b"null unique-id" in L.gsr_last_error()
    uid = ctypes.create_string_buffer(128)
    for world, rank in ((0, 0), (1, 1), (2, -1)):
        assert L.gsr_dp_init(uid, world, rank) != 0 and b"bad unique id" in L.gsr_last_error()
    assert L.gsr_dp_init(None, 1, 0) != 0
    assert L.gsr_dp_allreduce(None, 16, None) == -1 and b"null buffer" in L.gsr_last_error()
    assert L.gsr_dp_allreduce(None, 0, None) == -1 and b"not initialised" in L.gsr_last_error()
    assert L.gsr_dp_sh_exchange(10, 4, 16, 2, 16, 1, 16, 16, 16, None) == -1
    assert b"bad P / D / M / C" in L.gsr_last_error()
    assert L.gsr_dp_sh_exchange(10, 3, 16, 2, None, 1, 16, 16, 16, None) == -1
    assert b"null argument" in L.gsr_last_error()
    assert L.gsr_dp_sh_exchange(0, 3, 16, 2, None, 1, None, None, None, None) == -1
    assert b"not initialised" in L.gsr_last_error()
    for t in (-1, 0, 16):  # (the wait takes the lock and checks the communicator first)
        assert L.gsr_dp_wait(t, None) != 0 and b"not initialised" in L.gsr_last_error()


def test_deferred_forward_validates_without_the_device():
    """gsr_forward_deferred needs a binning buffer laid out for a capacity guess, and
    gsr_forward_wait only accepts a pending ticket: both fail cleanly before any device work."""
    from diff_gaussian_rasterization import _C
    L = ctypes.CDLL(_C.LIB_PATH)
    L.gsr_last_error.restype = ctypes.c_char_p
    t = ctypes.c_int(5)
    assert L.gsr_forward_deferred(None, None, None, None, None, ctypes.c_size_t(0), None, None, None, None, None,
                                  None, ctypes.byref(t)) != 0
    assert t.value == -1 and b"binning_capacity" in L.gsr_last_error()
    nr = ctypes.c_int(0)
    for bad in (0, -1, 999):
        assert L.gsr_forward_wait(bad, None, None, None, ctypes.byref(nr)) != 0
        assert b"not a pending ticket" in L.gsr_last_error()

