"""ctypes binding of libgsr.so (include/gsr.h) with the positional signatures of
the reference's private extension module `_C` (DGR/ext.cpp:15-19,
DGR/rasterize_points.h:18-73), so that the public API in __init__.py reads like
the reference's.

The product path is libgsr.so only: if it is missing, importing this module
raises ImportError -- there is no CPU or PyTorch fallback.
"""
import ctypes
import functools
import os

import torch  # must be imported first: libgsr.so binds to torch's HIP runtime (same soname)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GSR_LIBRARY", os.path.join(_HERE, "libgsr.so"))

if not os.path.exists(LIB_PATH):
    raise ImportError(
        f"libgsr.so not found at {LIB_PATH}; build it with "
        "`make -C 3d_gaussian_magic_change-segment_3dgs_amd/csrc` (or __graft_entry__.build())")

_lib = ctypes.CDLL(LIB_PATH)

NUM_CHANNELS = 3  # config.h:15
NUM_CLASS = 2     # config.h:16
ARENA_ALIGN = 64  # include/gsr_train.h GSR_ARENA_ALIGN (floats)


class _Settings(ctypes.Structure):
    _fields_ = [
        ("P", ctypes.c_int), ("D", ctypes.c_int), ("M", ctypes.c_int), ("W", ctypes.c_int), ("H", ctypes.c_int),
        ("tanfovx", ctypes.c_float), ("tanfovy", ctypes.c_float), ("scale_modifier", ctypes.c_float),
        ("prefiltered", ctypes.c_int), ("debug", ctypes.c_int),
        ("bg", ctypes.c_void_p), ("viewmatrix", ctypes.c_void_p), ("projmatrix", ctypes.c_void_p),
        ("campos", ctypes.c_void_p), ("binning_capacity", ctypes.c_int),
    ]


class _Inputs(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in (
        "means3D", "shs", "colors_precomp", "segments", "opacities", "scales", "rotations", "cov3D_precomp")]


class _Grads(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in (
        "dmeans2D", "dcolors", "dopacity", "dmeans3D", "dcov3D", "dsh", "dscales", "drot", "dsegments")]


_vp, _i, _sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
_lib.gsr_geom_bytes.restype = _sz
_lib.gsr_geom_bytes.argtypes = [_i]
_lib.gsr_binning_bytes.restype = _sz
_lib.gsr_binning_bytes.argtypes = [_i]
_lib.gsr_binning_capacity.restype = _i
_lib.gsr_binning_capacity.argtypes = [_sz]
_lib.gsr_img_bytes.restype = _sz
_lib.gsr_img_bytes.argtypes = [_i, _i]
_lib.gsr_backward_scratch_bytes.restype = _sz
_lib.gsr_backward_scratch_bytes.argtypes = [_i]
_lib.gsr_forward_geometry.restype = _i
_lib.gsr_forward_geometry.argtypes = [ctypes.POINTER(_Settings), ctypes.POINTER(_Inputs), _vp, _vp, _vp,
                                      ctypes.POINTER(ctypes.c_int)]
_lib.gsr_forward_render.restype = _i
_lib.gsr_forward_render.argtypes = [ctypes.POINTER(_Settings), ctypes.POINTER(_Inputs), _vp, _vp, _vp, _i,
                                    _vp, _vp, _vp, _vp, _vp]
_lib.gsr_forward.restype = _i
_lib.gsr_forward.argtypes = [ctypes.POINTER(_Settings), ctypes.POINTER(_Inputs), _vp, _vp, _vp, _sz, _vp,
                             _vp, _vp, _vp, _vp, _vp, ctypes.POINTER(ctypes.c_int)]
GSR_NEED_BINNING = 2
_lib.gsr_forward_deferred.restype = _i
_lib.gsr_forward_deferred.argtypes = [ctypes.POINTER(_Settings), ctypes.POINTER(_Inputs), _vp, _vp, _vp, _sz, _vp,
                                      _vp, _vp, _vp, _vp, _vp, ctypes.POINTER(ctypes.c_int)]
_lib.gsr_forward_wait.restype = _i
_lib.gsr_forward_wait.argtypes = [_i, ctypes.POINTER(_Settings), _vp, _vp, ctypes.POINTER(ctypes.c_int)]
_lib.gsr_backward.restype = _i
_lib.gsr_backward.argtypes = [ctypes.POINTER(_Settings), ctypes.POINTER(_Inputs), _vp, _vp, _vp, _vp, _i, _vp,
                              _vp, _vp, _vp, _vp, _vp, ctypes.POINTER(_Grads), _vp]
if hasattr(_lib, "gsr_backward_deferred_sh"):  # (absent from builds older than round 4: A/B runs)
    _lib.gsr_backward_deferred_sh.restype = _i
    _lib.gsr_backward_deferred_sh.argtypes = _lib.gsr_backward.argtypes[:-1] + [_vp, _vp]
_lib.gsr_mark_visible.restype = _i
_lib.gsr_mark_visible.argtypes = [_i, _vp, _vp, _vp, _vp, _vp]
_lib.gsr_last_error.restype = ctypes.c_char_p
_lib.gsr_version.restype = ctypes.c_char_p
_lib.gsr_debug_copy.restype = ctypes.c_longlong
_lib.gsr_debug_copy.argtypes = [ctypes.c_char_p, _i, _i, _i, _i, _i, _vp, _vp, _vp, _vp, _vp]

class _ViewState(ctypes.Structure):
    _fields_ = [("s", ctypes.POINTER(_Settings)), ("radii", ctypes.c_void_p), ("geom", ctypes.c_void_p),
                ("binning", ctypes.c_void_p), ("img", ctypes.c_void_p), ("num_rendered", ctypes.c_int),
                ("alpha", ctypes.c_void_p), ("dL_dcolor", ctypes.c_void_p), ("dL_dsegment", ctypes.c_void_p),
                ("dL_ddepth", ctypes.c_void_p), ("dL_dalpha", ctypes.c_void_p), ("scratch", ctypes.c_void_p),
                ("dmeans2D", ctypes.c_void_p)]


MAX_VIEWS = 16  # include/gsr.h GSR_MAX_VIEWS
_lib.gsr_multiview_scratch_bytes.restype = _sz
_lib.gsr_multiview_scratch_bytes.argtypes = [_i, _i]
_lib.gsr_backward_multiview.restype = _i
_lib.gsr_backward_multiview.argtypes = [_i, ctypes.POINTER(_ViewState), ctypes.POINTER(_Inputs), _vp,
                                        ctypes.POINTER(_Grads), _vp]

_lib.gsr_sh_rows_floats.restype = _sz
_lib.gsr_sh_rows_floats.argtypes = [_i]
_lib.gsr_backward_multiview_deferred_sh.restype = _i
_lib.gsr_backward_multiview_deferred_sh.argtypes = [_i, ctypes.POINTER(_ViewState), ctypes.POINTER(_Inputs), _vp,
                                                    ctypes.POINTER(_Grads), _vp]
_lib.gsr_sh_backward.restype = _i
_lib.gsr_sh_backward.argtypes = [_i, _i, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp]

_ll = ctypes.c_longlong
_lib.gsr_arena_layout.restype = _ll
_lib.gsr_arena_layout.argtypes = [_i, _i, _i, ctypes.POINTER(_ll)]
_lib.gsr_act_layout.restype = _ll
_lib.gsr_act_layout.argtypes = [_i, _i, ctypes.POINTER(_ll)]
_lib.gsr_set_option.restype = _i
_lib.gsr_set_option.argtypes = [ctypes.c_char_p, ctypes.c_longlong]
_lib.gsr_num_stages.restype = _i
_lib.gsr_stage_name.restype = ctypes.c_char_p
_lib.gsr_stage_name.argtypes = [_i]
_lib.gsr_timing_enable.argtypes = [_i]
_lib.gsr_timing_collect.restype = _i
_lib.gsr_timing_collect.argtypes = [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_longlong)]
_lib.gsr_stream_copy.restype = _i
_lib.gsr_stream_copy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, _i, ctypes.c_void_p]

# native data-parallel exchange (include/gsr.h, csrc/dp.hip): optional so that an older build
# without it still imports (gsr_tools.dp then keeps the torch.distributed path)
if hasattr(_lib, "gsr_dp_init"):
    _lib.gsr_dp_unique_id_bytes.restype = _sz
    _lib.gsr_dp_unique_id_bytes.argtypes = []
    _lib.gsr_dp_get_unique_id.restype = _i
    _lib.gsr_dp_get_unique_id.argtypes = [_vp]
    _lib.gsr_dp_init.restype = _i
    _lib.gsr_dp_init.argtypes = [_vp, _i, _i]
    _lib.gsr_dp_world.restype = _i
    _lib.gsr_dp_world.argtypes = []
    _lib.gsr_dp_finalize.restype = _i
    _lib.gsr_dp_finalize.argtypes = []
    _lib.gsr_dp_allreduce.restype = _i
    _lib.gsr_dp_allreduce.argtypes = [_vp, _sz, _vp]
    _lib.gsr_dp_sh_exchange.restype = _i
    _lib.gsr_dp_sh_exchange.argtypes = [_i, _i, _i, _i, _vp, _i, _vp, _vp, _vp, _vp]
    _lib.gsr_dp_wait.restype = _i
    _lib.gsr_dp_wait.argtypes = [_i, _vp]

EXPORTED_SYMBOLS = ("gsr_geom_bytes", "gsr_binning_bytes", "gsr_binning_capacity", "gsr_img_bytes", "gsr_backward_scratch_bytes",
                    "gsr_forward_geometry", "gsr_forward_render", "gsr_forward", "gsr_forward_deferred",
                    "gsr_forward_wait", "gsr_backward", "gsr_mark_visible",
                    "gsr_debug_copy", "gsr_num_stages", "gsr_stage_name", "gsr_timing_enable", "gsr_timing_collect",
                    "gsr_stream_copy",
                    "gsr_last_error", "gsr_version", "gsr_set_option", "gsr_multiview_scratch_bytes",
                    "gsr_backward_multiview", "gsr_sh_rows_floats", "gsr_backward_multiview_deferred_sh",
                    "gsr_sh_backward", "gsr_backward_deferred_sh", "gsr_dp_unique_id_bytes", "gsr_dp_get_unique_id",
                    "gsr_dp_init", "gsr_dp_world", "gsr_dp_finalize", "gsr_dp_allreduce", "gsr_dp_sh_exchange",
                    "gsr_dp_wait")

_DEBUG_FIELDS = {  # name -> (dtype, elements per unit, unit: P | I | T)
    "tiles_touched": (torch.int32, 1, "P"), "rec": (torch.float32, 16, "P"), "clamped": (torch.uint8, 1, "P"),
    "order": (torch.int32, 1, "P"), "goff": (torch.int32, 1, "P"), "bbase": (torch.int32, 1, "P/256"),
    "point_list": (torch.int32, 1, "I"),
    "slot_vals": (torch.int32, 1, "I"), "ranges": (torch.int32, 2, "T"), "n_contrib_tiles": (torch.int32, 256, "T"),
    "written": (torch.uint8, 1, "I"),  # after a backward: 1 where the render backward stored a record
    "tile_order": (torch.int32, 1, "T+"),  # heavy-first tile order + the render schedule (gsr_internal.h TileSched)
}


def debug_state(name, P, W, H, num_rendered, geomBuffer, binningBuffer, imgBuffer):
    """Copy of one private intermediate of a forward call (parity tests only; see
    gsr_debug_copy in include/gsr.h).  Unsigned arrays are returned as int32."""
    dtype, per, unit = _DEBUG_FIELDS[name]
    T = ((W + 15) // 16) * ((H + 15) // 16)
    if unit == "T+":  # the schedule's length is the library's (gsr_internal.h TileSched): ask it
        nb = int(_lib.gsr_debug_copy(name.encode(), P, W, H, num_rendered, 0, None, None, None, None, None))
        if nb < 0:
            raise RuntimeError(f"gsr_debug_copy({name}) size query failed: {_lib.gsr_last_error().decode()}")
        n = nb // 4
    else:
        n = {"P": P, "P/256": (P + 255) // 256, "I": num_rendered, "T": T}[unit] * per
    dev = geomBuffer.device
    out = torch.empty(max(n, 1), dtype=dtype, device=dev)
    ptr = lambda t: t.data_ptr() if t is not None and t.numel() else None
    rc = _lib.gsr_debug_copy(name.encode(), P, W, H, num_rendered, binning_capacity(binningBuffer),
                             ptr(geomBuffer), ptr(binningBuffer), ptr(imgBuffer), out.data_ptr(), _stream(dev))
    if rc < 0:
        raise RuntimeError(f"gsr_debug_copy({name}) failed: {_lib.gsr_last_error().decode()}")
    return out[:n]


def binning_capacity(binning):
    """Layout capacity (instances) of a binning buffer allocated as gsr_binning_bytes(C)
    (gsr_settings.binning_capacity; 0 for an empty buffer)."""
    if binning is None or binning.numel() == 0:
        return 0
    return max(0, int(_lib.gsr_binning_capacity(binning.numel())))


def version():
    return _lib.gsr_version().decode()


def _check(rc):
    if rc != 0:
        raise RuntimeError(_lib.gsr_last_error().decode())


def _present(t):
    return isinstance(t, torch.Tensor) and t.numel() > 0


def _dev_f32(t, device, name, align=4):
    """Contiguous fp32 tensor on `device` (reference: .contiguous().data<float>()),
    re-allocated if its address is not `align`-aligned for vector loads."""
    if not _present(t):
        return None
    if t.dtype != torch.float32:
        raise RuntimeError(f"{name} must be a float32 tensor (got {t.dtype})")
    if t.device != device:
        if t.device.type != "cpu":
            raise RuntimeError(f"{name} is on {t.device}, expected {device}")
        t = t.to(device)
    t = t.contiguous()
    if t.data_ptr() % align:
        t = t.clone()
    return t


_BIN_GUESS = os.environ.get("GSR_BIN_GUESS", "1") != "0"
# the single-view host work in C++ when built (_host.py; None: this module's ctypes route)
from . import _host  # noqa: E402
_HOST = _host.load()
# the single-view autograd function in C++ as well (RasterizeFn; GSR_HOST_AUTOGRAD=0: the Python
# _RasterizeGaussians over _HOST, A/B of the host overhead)
_HOST_AUTOGRAD = _HOST if _HOST is not None and os.environ.get("GSR_HOST_AUTOGRAD", "1") != "0" else None
_last_rendered = {}  # device -> num_rendered of the recent forwards (binning size guess)
_GUESS_WINDOW = 16   # a trainer cycling through a batch of views sees each view's count again


def _ptr(t):
    return None if t is None else t.data_ptr()


def _stream(device):
    return torch.cuda.current_stream(device).cuda_stream


def _settings(P, D, M, W, H, tanfovx, tanfovy, scale_modifier, prefiltered, debug, bg, view, proj, campos):
    s = _Settings()
    s.P, s.D, s.M, s.W, s.H = P, D, M, W, H
    s.tanfovx, s.tanfovy, s.scale_modifier = float(tanfovx), float(tanfovy), float(scale_modifier)
    s.prefiltered, s.debug = int(bool(prefiltered)), int(bool(debug))
    s.bg, s.viewmatrix, s.projmatrix, s.campos = _ptr(bg), _ptr(view), _ptr(proj), _ptr(campos)
    return s


def _inputs(means3D, sh, colors, segments, opacity, scales, rotations, cov3D_precomp):
    i = _Inputs()
    i.means3D, i.shs, i.colors_precomp, i.segments = _ptr(means3D), _ptr(sh), _ptr(colors), _ptr(segments)
    i.opacities, i.scales, i.rotations, i.cov3D_precomp = _ptr(opacity), _ptr(scales), _ptr(rotations), _ptr(
        cov3D_precomp)
    return i


def _check_segments(segments, P):
    if segments is not None and (segments.dim() != 2 or segments.shape[1] != NUM_CLASS or segments.shape[0] != P):
        raise RuntimeError(f"segments must have shape (num_points, {NUM_CLASS}) (reference config.h:16 NUM_CLASS)")


def _guess(device):
    """Binning capacity guess for the next forward on `device`: the largest of the recent
    counts + 15% (0: none)."""
    recent = _last_rendered.get(device)
    cap = max(recent) if recent else 0
    return cap + cap // 7 + 4096 if cap and _BIN_GUESS else 0


def _record(device, num_rendered):
    recent = _last_rendered.setdefault(device, [])
    recent.append(num_rendered)
    del recent[:-_GUESS_WINDOW]


def last_num_rendered(device):
    """num_rendered of the latest single-view forward with P > 0 on `device` (every route records
    it; the C++ autograd route's graph node carries no Python attributes)."""
    return _last_rendered[device][-1]


def rasterize_gaussians(background, means3D, colors, segments, opacity, scales, rotations, scale_modifier,
                        cov3D_precomp, viewmatrix, projmatrix, tan_fovx, tan_fovy, image_height, image_width, sh,
                        degree, campos, prefiltered, debug):
    """RasterizeGaussiansCUDA (DGR/rasterize_points.cu:35-125).
    Returns (num_rendered, color, depth, segment, alpha, radii, geomBuffer, binningBuffer, imgBuffer)."""
    if _HOST is not None:  # the same work in C++ (csrc/host_ext.cpp)
        device = means3D.device
        out = _HOST.rasterize_gaussians(background, means3D, colors, segments, opacity, scales, rotations,
                                        float(scale_modifier), cov3D_precomp, viewmatrix, projmatrix, float(tan_fovx),
                                        float(tan_fovy), int(image_height), int(image_width), sh, int(degree), campos,
                                        bool(prefiltered), bool(debug), _guess(device))
        if means3D.size(0) > 0:
            _record(device, out[0])
        return out
    return rasterize_gaussians_end(_forward_begin(False, background, means3D, colors, segments, opacity, scales,
                                                  rotations, scale_modifier, cov3D_precomp, viewmatrix, projmatrix,
                                                  tan_fovx, tan_fovy, image_height, image_width, sh, degree, campos,
                                                  prefiltered, debug))


# GSR_MV_DEFERRED=0: rasterize_gaussians_begin waits like rasterize_gaussians (A/B of the deferred forward)
_DEFERRED = os.environ.get("GSR_MV_DEFERRED", "1") != "0"


def rasterize_gaussians_begin(*args):
    """rasterize_gaussians split for a batch of views (same arguments): launches the view's
    forward and returns a handle at once when a binning-capacity guess exists
    (gsr_forward_deferred), so that the next views' launches do not wait for this view's
    num_rendered; rasterize_gaussians_end(handle), called on the same stream, waits and returns
    rasterize_gaussians' tuple.  Every handle must be ended (at most GSR_MAX_DEFERRED = 16
    open per thread)."""
    return _forward_begin(_DEFERRED, *args)


def _forward_begin(deferred, background, means3D, colors, segments, opacity, scales, rotations, scale_modifier,
                   cov3D_precomp, viewmatrix, projmatrix, tan_fovx, tan_fovy, image_height, image_width, sh,
                   degree, campos, prefiltered, debug):
    if means3D.dim() != 2 or means3D.size(1) != 3:
        raise RuntimeError("means3D must have dimensions (num_points, 3)")
    P, H, W = int(means3D.size(0)), int(image_height), int(image_width)
    device = means3D.device
    if device.type != "cuda":
        raise RuntimeError("gsr rasterizer: means3D must be a GPU tensor (the HIP path has no CPU fallback)")
    with torch.cuda.device(device):
        f32 = dict(dtype=torch.float32, device=device)
        if P == 0:  # reference leaves the zero-filled outputs untouched (rasterize_points.cu:87)
            z = lambda *s: torch.zeros(*s, **f32)
            empty = torch.empty(0, dtype=torch.uint8, device=device)
            return {"result": (0, z(NUM_CHANNELS, H, W), z(1, H, W), z(NUM_CLASS, H, W), z(1, H, W),
                               torch.zeros(0, dtype=torch.int32, device=device), empty, empty.clone(),
                               empty.clone())}
        means3D_ = _dev_f32(means3D, device, "means3D")
        sh_ = _dev_f32(sh, device, "sh")
        colors_ = _dev_f32(colors, device, "colors_precomp")
        segments_ = _dev_f32(segments, device, "segments", align=8)
        _check_segments(segments_, P)
        opacity_ = _dev_f32(opacity, device, "opacities")
        scales_ = _dev_f32(scales, device, "scales")
        rotations_ = _dev_f32(rotations, device, "rotations", align=16)
        cov_ = _dev_f32(cov3D_precomp, device, "cov3D_precomp")
        bg_ = _dev_f32(background, device, "bg")
        view_ = _dev_f32(viewmatrix, device, "viewmatrix")
        proj_ = _dev_f32(projmatrix, device, "projmatrix")
        campos_ = _dev_f32(campos, device, "campos")
        M = int(sh_.size(1)) if sh_ is not None else 0
        s = _settings(P, int(degree), M, W, H, tan_fovx, tan_fovy, scale_modifier, prefiltered, debug, bg_, view_,
                      proj_, campos_)
        inp = _inputs(means3D_, sh_, colors_, segments_, opacity_, scales_, rotations_, cov_)
        stream = _stream(device)
        u8 = dict(dtype=torch.uint8, device=device)
        geom = torch.empty(_lib.gsr_geom_bytes(P), **u8)
        img = torch.empty(_lib.gsr_img_bytes(W, H), **u8)
        radii = torch.empty(P, dtype=torch.int32, device=device)
        # outputs are allocated before the num_rendered sync so that only the binning
        # buffer is allocated between the sync and the render launches
        color = torch.empty(NUM_CHANNELS, H, W, **f32)
        depth = torch.empty(1, H, W, **f32)
        alpha = torch.empty(1, H, W, **f32)
        segment = torch.empty(NUM_CLASS, H, W, **f32)
        # The binning buffer depends on num_rendered, known only after the geometry
        # stage; allocate a guess (the largest of the recent counts on this device + 15%)
        # before it so that nothing but the render launches sits between the sync and the
        # GPU.  The largest, not the last: consecutive calls of a multi-view batch render
        # different views, and a guess below the count costs an exact re-run of stage B.
        cap = _guess(device)
        binning = torch.empty(_lib.gsr_binning_bytes(cap), **u8) if cap else None
        # every call on a binning buffer uses the layout of its capacity (gsr.h); with a guess
        # gsr_forward runs stage B speculatively right behind stage A
        s.binning_capacity = binning_capacity(binning)
        h = {"s": s, "inp": inp, "stream": stream, "device": device, "geom": geom, "img": img, "radii": radii,
             "color": color, "depth": depth, "alpha": alpha, "segment": segment, "binning": binning,
             # the device inputs the launches read stay referenced until the handle is ended
             "keep": (means3D_, sh_, colors_, segments_, opacity_, scales_, rotations_, cov_, bg_, view_, proj_,
                      campos_)}
        bptr = binning.data_ptr() if binning is not None else None
        bbytes = binning.numel() if binning is not None else 0
        if deferred and cap and not debug:
            t = ctypes.c_int(-1)
            _check(_lib.gsr_forward_deferred(ctypes.byref(s), ctypes.byref(inp), geom.data_ptr(), radii.data_ptr(),
                                             bptr, bbytes, img.data_ptr(), color.data_ptr(), depth.data_ptr(),
                                             alpha.data_ptr(), segment.data_ptr(), stream, ctypes.byref(t)))
            h["ticket"] = t.value
            return h
        nr = ctypes.c_int(0)
        # geometry, the num_rendered sync and the render in one C call when the guess holds
        h["rc"] = _lib.gsr_forward(ctypes.byref(s), ctypes.byref(inp), geom.data_ptr(), radii.data_ptr(), bptr,
                                   bbytes, img.data_ptr(), color.data_ptr(), depth.data_ptr(), alpha.data_ptr(),
                                   segment.data_ptr(), stream, ctypes.byref(nr))
        h["num_rendered"] = int(nr.value)
        return h


def rasterize_gaussians_end(h):
    """Completes a rasterize_gaussians_begin handle (see there)."""
    if "result" in h:
        return h["result"]
    s, device, stream = h["s"], h["device"], h["stream"]
    with torch.cuda.device(device):
        if "ticket" in h:
            nr = ctypes.c_int(0)
            rc = _lib.gsr_forward_wait(h.pop("ticket"), ctypes.byref(s), h["geom"].data_ptr(), stream,
                                       ctypes.byref(nr))
            num_rendered = int(nr.value)
        else:
            rc, num_rendered = h["rc"], h["num_rendered"]
        _record(device, num_rendered)
        binning = h["binning"]
        if rc == GSR_NEED_BINNING:  # no guess, or too small: stage B with the exact size
            binning = torch.empty(_lib.gsr_binning_bytes(num_rendered), dtype=torch.uint8, device=device)
            s.binning_capacity = binning_capacity(binning)
            rc = _lib.gsr_forward_render(ctypes.byref(s), ctypes.byref(h["inp"]), h["geom"].data_ptr(),
                                         binning.data_ptr(), h["img"].data_ptr(), num_rendered,
                                         h["color"].data_ptr(), h["depth"].data_ptr(), h["alpha"].data_ptr(),
                                         h["segment"].data_ptr(), stream)
        _check(rc)
        if binning is None:  # num_rendered == 0 with no guess
            binning = torch.empty(0, dtype=torch.uint8, device=device)
    return (num_rendered, h["color"], h["depth"], h["segment"], h["alpha"], h["radii"], h["geom"], binning,
            h["img"])


def set_option(name, value):
    """Process-wide tuning / test hook (include/gsr.h: gsr_set_option)."""
    _check(_lib.gsr_set_option(name.encode(), int(value)))


# Tuning experiments without a rebuild: GSR_OPTIONS="name=value,name=value" is applied at
# import (e.g. GSR_OPTIONS="split_fwd_bucket=10,split_bwd_depth=0").  A malformed or unknown
# entry is reported and skipped: a typo in an environment variable must not break the import.
for _kv in filter(None, (e.strip() for e in os.environ.get("GSR_OPTIONS", "").split(","))):
    try:
        _k, _v = _kv.split("=")
        set_option(_k.strip(), int(_v))
    except (ValueError, RuntimeError) as _e:
        import warnings
        warnings.warn(f"GSR_OPTIONS entry {_kv!r} ignored: {_e}")


@functools.lru_cache(maxsize=64)
def grad_arena_layout(P, M):
    """Offsets (in floats) of the gradients inside the single arena allocated by
    rasterize_gaussians_backward.  The first `bucket` floats are the parameter
    gradients a data-parallel trainer all-reduces: [dmeans3D | dsh | dopacity |
    dscales | drot | dsegments], laid out exactly like the
    training arena of include/gsr_train.h (every block 64-float aligned), so the
    bucket is also the gradient of the trainer's parameter arena; means2D /
    colour / cov3D grads follow.  Maps name -> (offset, floats per Gaussian)."""
    off = (ctypes.c_longlong * 7)()
    _lib.gsr_arena_layout(P, M, NUM_CLASS, off)
    names = [("dmeans3D", 3), ("dsh", 3 * M), ("dopacity", 1), ("dscales", 3), ("drot", 4),
             ("dsegments", NUM_CLASS)]
    lay = {n: (int(off[b]), k) for b, (n, k) in enumerate(names)}
    lay["bucket"] = (0, int(off[6]))
    o = int(off[6])
    for n, k in (("dmeans2D", 3), ("dcolors", 3), ("dcov3D", 6)):
        lay[n] = (o, k)
        o += -(-k * P // ARENA_ALIGN) * ARENA_ALIGN
    lay["total"] = (0, o)
    return lay


def rasterize_gaussians_backward(background, means3D, radii, colors, segments, scales, rotations, scale_modifier,
                                 cov3D_precomp, viewmatrix, projmatrix, tan_fovx, tan_fovy, dL_dout_color,
                                 dL_dout_segment, dL_dout_depth, dL_dout_alpha, sh, degree, campos, geomBuffer, R,
                                 binningBuffer, imageBuffer, alpha, debug, sh_rows=None):
    """RasterizeGaussiansBackwardCUDA (DGR/rasterize_points.cu:127-221).
    sh_rows (fp32 tensor of sh_rows_floats(P) on the GPU, 16-B aligned): deferred SH mode
    (gsr_backward_deferred_sh) -- this view's SH exchange rows are written there and the
    returned dsh is left unwritten until sh_backward completes it.
    Returns (dL_dmeans2D, dL_dcolors, dL_dopacity, dL_dmeans3D, dL_dcov3D, dL_dsh, dL_dscales,
    dL_drotations, dL_dsegments).  Gradients of absent (empty) inputs are zero tensors of the
    reference's shapes ([P,3] / [P,6] / [P,0,3] / [P,3] / [P,4] / [P,2], rasterize_points.cu:
    166-177), as read-only stride-0 views of one zero (no memory traffic)."""
    if _HOST is not None and sh_rows is None:  # the same work in C++ (csrc/host_ext.cpp)
        return _HOST.rasterize_gaussians_backward(background, means3D, radii, colors, segments, scales, rotations,
                                                  float(scale_modifier), cov3D_precomp, viewmatrix, projmatrix,
                                                  float(tan_fovx), float(tan_fovy), dL_dout_color, dL_dout_segment,
                                                  dL_dout_depth, dL_dout_alpha, sh, int(degree), campos, geomBuffer,
                                                  int(R), binningBuffer, imageBuffer, alpha, bool(debug))
    P = int(means3D.size(0))
    shaped = next(t for t in (dL_dout_color, dL_dout_segment, dL_dout_depth, dL_dout_alpha, alpha) if t is not None)
    H, W = int(shaped.size(-2)), int(shaped.size(-1))
    device = means3D.device
    with torch.cuda.device(device):
        means3D_ = _dev_f32(means3D, device, "means3D")
        sh_ = _dev_f32(sh, device, "sh")
        colors_ = _dev_f32(colors, device, "colors_precomp")
        segments_ = _dev_f32(segments, device, "segments", align=8)
        scales_ = _dev_f32(scales, device, "scales")
        rotations_ = _dev_f32(rotations, device, "rotations", align=16)
        cov_ = _dev_f32(cov3D_precomp, device, "cov3D_precomp")
        M = int(sh_.size(1)) if sh_ is not None else 0
        lay = grad_arena_layout(P, M)
        arena = torch.empty(lay["total"][1], dtype=torch.float32, device=device)

        def view(name, *shape):
            o, k = lay[name]
            return arena.narrow(0, o, k * P).view(P, *shape)

        dmeans3D, dsh, dopacity = view("dmeans3D", 3), view("dsh", M, 3), view("dopacity", 1)
        dscales, drot, dsegments = view("dscales", 3), view("drot", 4), view("dsegments", NUM_CLASS)
        dmeans2D, dcolors, dcov3D = view("dmeans2D", 3), view("dcolors", 3), view("dcov3D", 6)
        if P == 0:
            arena.zero_()
            return dmeans2D, dcolors, dopacity, dmeans3D, dcov3D, dsh, dscales, drot, dsegments
        bg_ = _dev_f32(background, device, "bg")
        view_ = _dev_f32(viewmatrix, device, "viewmatrix")
        proj_ = _dev_f32(projmatrix, device, "projmatrix")
        campos_ = _dev_f32(campos, device, "campos")
        s = _settings(P, int(degree), M, W, H, tan_fovx, tan_fovy, scale_modifier, False, debug, bg_, view_, proj_,
                      campos_)
        s.binning_capacity = binning_capacity(binningBuffer)
        inp = _inputs(means3D_, sh_, colors_, segments_, None, scales_, rotations_, cov_)  # opacities unused
        ups = [_dev_f32(t, device, n) for t, n in ((dL_dout_color, "dL_dcolor"), (dL_dout_segment, "dL_dsegment"),
                                                   (dL_dout_depth, "dL_ddepth"), (dL_dout_alpha, "dL_dalpha"))]
        ups = [u if u is not None else torch.zeros(c, H, W, dtype=torch.float32, device=device)
               for u, c in zip(ups, (NUM_CHANNELS, NUM_CLASS, 1, 1))]
        alpha_ = _dev_f32(alpha, device, "alpha")
        radii_ = radii.contiguous()
        R = int(R)
        scratch = torch.empty(_lib.gsr_backward_scratch_bytes(R), dtype=torch.uint8, device=device)
        g = _Grads()
        g.dmeans2D, g.dopacity, g.dmeans3D = dmeans2D.data_ptr(), dopacity.data_ptr(), dmeans3D.data_ptr()
        g.dcolors = dcolors.data_ptr() if colors_ is not None else None
        g.dcov3D = dcov3D.data_ptr() if cov_ is not None else None
        g.dsh = dsh.data_ptr() if (sh_ is not None and M > 0) else None
        g.dscales = dscales.data_ptr() if scales_ is not None else None
        g.drot = drot.data_ptr() if scales_ is not None else None
        g.dsegments = dsegments.data_ptr()
        bargs = (ctypes.byref(s), ctypes.byref(inp), radii_.data_ptr(), geomBuffer.data_ptr(),
                 binningBuffer.data_ptr() if binningBuffer.numel() else None, imageBuffer.data_ptr(), R,
                 alpha_.data_ptr(), ups[0].data_ptr(), ups[1].data_ptr(), ups[2].data_ptr(), ups[3].data_ptr(),
                 scratch.data_ptr() if R > 0 else None, ctypes.byref(g))
        if sh_rows is not None:
            if sh_ is None:
                raise RuntimeError("deferred SH backward: sh is required")
            if (sh_rows.device != device or sh_rows.dtype != torch.float32 or not sh_rows.is_contiguous()
                    or sh_rows.numel() < sh_rows_floats(P) or sh_rows.data_ptr() % 16):
                raise RuntimeError("deferred SH backward: sh_rows must be a contiguous, 16-B aligned float32 "
                                   f"tensor of sh_rows_floats(P) floats on {device}")
            _check(_lib.gsr_backward_deferred_sh(*bargs, sh_rows.data_ptr(), _stream(device)))
        else:
            _check(_lib.gsr_backward(*bargs, _stream(device)))
    Z = lambda *shape: _zeros(device, *shape)
    return (dmeans2D, dcolors if colors_ is not None else Z(P, 3), dopacity, dmeans3D,
            dcov3D if cov_ is not None else Z(P, 6), dsh if sh_ is not None else Z(P, 0, 3),
            dscales if scales_ is not None else Z(P, 3), drot if scales_ is not None else Z(P, 4),
            dsegments if segments_ is not None else Z(P, NUM_CLASS))


_ZERO = {}


def _zeros(device, *shape):
    """A zero-filled [shape] tensor without memory traffic: one cached zero, expanded."""
    z = _ZERO.get(device)
    if z is None:
        z = _ZERO[device] = torch.zeros((), dtype=torch.float32, device=device)
    return z.expand(*shape)


def mark_visible(means3D, viewmatrix, projmatrix):
    """markVisible (DGR/rasterize_points.cu:223-242): bool [P]."""
    P = int(means3D.size(0))
    device = means3D.device
    with torch.cuda.device(device):
        present = torch.zeros(P, dtype=torch.bool, device=device)
        if P == 0:
            return present
        m = _dev_f32(means3D, device, "means3D")
        v = _dev_f32(viewmatrix, device, "viewmatrix")
        p = _dev_f32(projmatrix, device, "projmatrix")
        _check(_lib.gsr_mark_visible(P, m.data_ptr(), v.data_ptr(), p.data_ptr(), present.data_ptr(),
                                     _stream(device)))
    return present


def sh_rows_floats(P):
    """Floats of one view's SH exchange rows (include/gsr.h gsr_sh_rows_floats)."""
    return int(_lib.gsr_sh_rows_floats(int(P)))


def sh_backward(sh_rows, V, means3D, sh, degree, dsh, dmeans3D):
    """gsr_sh_backward: from V views' SH exchange rows (sh_rows: fp32, V x
    sh_rows_floats(P), on the GPU), write dsh [P,M,3] = sum over the views of
    basis x dRGB.  The views' SH direction terms are already in dmeans3D (each rank
    adds its own in the multi-view backward); `sh` gives M and `dmeans3D` is not
    touched (both kept for the signature)."""
    P = int(means3D.size(0))
    M = int(sh.size(1))
    device = means3D.device
    for t, n in ((sh_rows, "sh_rows"), (means3D, "means3D"), (sh, "sh"), (dsh, "dsh"), (dmeans3D, "dmeans3D")):
        if t is not None and (t.device != device or t.dtype != torch.float32 or not t.is_contiguous()):
            raise RuntimeError(f"sh_backward: {n} must be a contiguous float32 tensor on {device}")
    if sh_rows.numel() < int(V) * sh_rows_floats(P):
        raise RuntimeError("sh_backward: sh_rows holds fewer than V views")
    with torch.cuda.device(device):
        _check(_lib.gsr_sh_backward(int(V), P, int(degree), M, sh.data_ptr(), means3D.data_ptr(),
                                    sh_rows.data_ptr(), _ptr(dsh), _ptr(dmeans3D), _stream(device)))


def rasterize_gaussians_backward_multiview(views, means3D, colors, segments, scales, rotations, scale_modifier,
                                           cov3D_precomp, sh, degree, debug, sh_rows=None):
    """gsr_backward_multiview: the summed parameter gradients of several views.
    `views` holds, per view, the raster settings fields (bg, viewmatrix, projmatrix,
    tanfovx, tanfovy, image_height, image_width, campos), the forward state
    (radii, geom, binning, img, num_rendered, alpha) and the upstream gradients
    (dL_dcolor, dL_dsegment, dL_ddepth, dL_dalpha; None = zeros).  Returns the
    single-view tuple (dmeans2D = None, dcolors, dopacity, dmeans3D, dcov3D, dsh,
    dscales, drot, dsegments) -- one gradient arena, bucket first -- and the list of
    per-view dmeans2D [P,3].

    sh_rows (fp32 tensor of B x sh_rows_floats(P) on the GPU, 16-B aligned): deferred
    SH mode (gsr_backward_multiview_deferred_sh) -- the views' SH exchange rows are
    written there, dsh is left unwritten and dmeans3D lacks the SH direction term
    until sh_backward completes them (after a view-parallel exchange)."""
    B = len(views)
    if not 1 <= B <= MAX_VIEWS:
        raise RuntimeError(f"multiview backward: 1..{MAX_VIEWS} views per call")
    P = int(means3D.size(0))
    device = means3D.device
    with torch.cuda.device(device):
        means3D_ = _dev_f32(means3D, device, "means3D")
        sh_ = _dev_f32(sh, device, "sh")
        colors_ = _dev_f32(colors, device, "colors_precomp")
        segments_ = _dev_f32(segments, device, "segments", align=8)
        scales_ = _dev_f32(scales, device, "scales")
        rotations_ = _dev_f32(rotations, device, "rotations", align=16)
        cov_ = _dev_f32(cov3D_precomp, device, "cov3D_precomp")
        M = int(sh_.size(1)) if sh_ is not None else 0
        lay = grad_arena_layout(P, M)
        arena = torch.empty(lay["total"][1], dtype=torch.float32, device=device)

        def view_(name, *shape):
            o, k = lay[name]
            return arena.narrow(0, o, k * P).view(P, *shape)

        dmeans3D, dsh, dopacity = view_("dmeans3D", 3), view_("dsh", M, 3), view_("dopacity", 1)
        dscales, drot, dsegments = view_("dscales", 3), view_("drot", 4), view_("dsegments", NUM_CLASS)
        dcolors, dcov3D = view_("dcolors", 3), view_("dcov3D", 6)
        f32 = dict(dtype=torch.float32, device=device)
        d2 = [torch.empty(P, 3, **f32) for _ in range(B)]
        out = (None, dcolors if colors_ is not None else None, dopacity, dmeans3D,
               dcov3D if cov_ is not None else None, dsh if sh_ is not None else None,
               dscales if scales_ is not None else None, drot if scales_ is not None else None,
               dsegments if segments_ is not None else None)
        if P == 0:
            arena.zero_()
            return out, d2
        keep = []  # ctypes structs and converted tensors must outlive the call
        states = (_ViewState * B)()
        for v, V in enumerate(views):
            H, W = int(V["image_height"]), int(V["image_width"])
            bg_ = _dev_f32(V["bg"], device, "bg")
            vm = _dev_f32(V["viewmatrix"], device, "viewmatrix")
            pm = _dev_f32(V["projmatrix"], device, "projmatrix")
            cp = _dev_f32(V["campos"], device, "campos")
            st = _settings(P, int(degree), M, W, H, V["tanfovx"], V["tanfovy"], scale_modifier, False, debug, bg_,
                           vm, pm, cp)
            st.binning_capacity = binning_capacity(V["binning"])
            ups = [_dev_f32(V[n], device, n) for n in ("dL_dcolor", "dL_dsegment", "dL_ddepth", "dL_dalpha")]
            ups = [u if u is not None else torch.zeros(c, H, W, **f32)
                   for u, c in zip(ups, (NUM_CHANNELS, NUM_CLASS, 1, 1))]
            alpha_ = _dev_f32(V["alpha"], device, "alpha")
            R = int(V["num_rendered"])
            scratch = torch.empty(_lib.gsr_backward_scratch_bytes(R), dtype=torch.uint8, device=device)
            radii_ = V["radii"].contiguous()
            keep += [st, bg_, vm, pm, cp, ups, alpha_, scratch, radii_]
            S = states[v]
            S.s = ctypes.pointer(st)
            S.radii, S.geom = radii_.data_ptr(), V["geom"].data_ptr()
            S.binning = V["binning"].data_ptr() if V["binning"].numel() else None
            S.img, S.num_rendered, S.alpha = V["img"].data_ptr(), R, alpha_.data_ptr()
            S.dL_dcolor, S.dL_dsegment, S.dL_ddepth, S.dL_dalpha = (u.data_ptr() for u in ups)
            S.scratch = scratch.data_ptr() if R > 0 else None
            S.dmeans2D = d2[v].data_ptr()
        inp = _inputs(means3D_, sh_, colors_, segments_, None, scales_, rotations_, cov_)
        mv = torch.empty(_lib.gsr_multiview_scratch_bytes(P, B) if sh_rows is None else 1, dtype=torch.uint8,
                         device=device)
        g = _Grads()
        g.dmeans2D, g.dopacity, g.dmeans3D = None, dopacity.data_ptr(), dmeans3D.data_ptr()
        g.dcolors = dcolors.data_ptr() if colors_ is not None else None
        g.dcov3D = dcov3D.data_ptr() if cov_ is not None else None
        g.dsh = dsh.data_ptr() if (sh_ is not None and M > 0) else None
        g.dscales = dscales.data_ptr() if scales_ is not None else None
        g.drot = drot.data_ptr() if scales_ is not None else None
        g.dsegments = dsegments.data_ptr()
        if sh_rows is not None:
            if sh_ is None:
                raise RuntimeError("deferred SH backward needs SH coefficients (shs)")
            if (sh_rows.device != device or sh_rows.dtype != torch.float32 or not sh_rows.is_contiguous()
                    or sh_rows.numel() < B * sh_rows_floats(P) or sh_rows.data_ptr() % 16):
                raise RuntimeError("sh_rows must be a contiguous, 16-B aligned float32 GPU tensor of "
                                   "B x sh_rows_floats(P) floats")
            _check(_lib.gsr_backward_multiview_deferred_sh(B, states, ctypes.byref(inp), sh_rows.data_ptr(),
                                                           ctypes.byref(g), _stream(device)))
        else:
            _check(_lib.gsr_backward_multiview(B, states, ctypes.byref(inp), mv.data_ptr(), ctypes.byref(g),
                                               _stream(device)))
    return out, d2
