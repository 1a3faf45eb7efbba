"""ctypes binding of the training-step entry points of libgsr.so
(include/gsr_train.h) and the arena layout they share with the rasterizer's
gradient arena.  Same library and loading rule as diff_gaussian_rasterization._C:
no CPU or PyTorch fallback -- a missing libgsr.so raises at import."""
import ctypes

import torch

from diff_gaussian_rasterization._C import _lib, _check, _stream, NUM_CLASS, ARENA_ALIGN  # noqa: F401

_vp, _i, _ll = ctypes.c_void_p, ctypes.c_int, ctypes.c_longlong

ADAM_GROUPS = 7
# Reference param-group order (scene/gaussian_model.py:162-170).
GROUP_NAMES = ("xyz", "f_dc", "f_rest", "opacity", "segment", "scaling", "rotation")
BLOCK_NAMES = ("xyz", "features", "opacity", "scaling", "rotation", "segment")  # arena block order


class AdamHyper(ctypes.Structure):
    _fields_ = [("beta1", ctypes.c_float), ("beta2", ctypes.c_float), ("eps", ctypes.c_float),
                ("one_minus_beta1", ctypes.c_float), ("one_minus_beta2", ctypes.c_float),
                ("step_size", ctypes.c_float * ADAM_GROUPS), ("bc2_sqrt", ctypes.c_float * ADAM_GROUPS),
                ("skip", ctypes.c_int * ADAM_GROUPS)]


_lib.gsr_activate.restype = _i
_lib.gsr_activate.argtypes = [_i, _i, _i, _vp, _vp, _vp]
_lib.gsr_activation_backward.restype = _i
_lib.gsr_activation_backward.argtypes = [_i, _i, _i, _vp, _vp, _vp, _vp]
_lib.gsr_adam_step.restype = _i
_lib.gsr_adam_step.argtypes = [_i, _i, _i, _vp, _vp, _vp, _vp, _vp, ctypes.POINTER(AdamHyper), _vp]
_lib.gsr_densify_stats.restype = _i
_lib.gsr_densify_stats.argtypes = [_i, _vp, _vp, _vp, _vp, _vp, _vp, _vp]

DENSIFY_AND_PRUNE, PRUNE_MASK, CLONE_ONLY, SPLIT_ONLY = 0, 1, 2, 3


class DensifyArgs(ctypes.Structure):
    _fields_ = [("mode", ctypes.c_int), ("split_n", ctypes.c_int), ("max_grad", ctypes.c_float),
                ("min_opacity", ctypes.c_float), ("clone_max_scale", ctypes.c_float),
                ("prune_max_scale", ctypes.c_float), ("max_screen_size", ctypes.c_float),
                ("split_divisor", ctypes.c_float)]


_lib.gsr_densify_ws_bytes.restype = ctypes.c_size_t
_lib.gsr_densify_ws_bytes.argtypes = [_i]
_lib.gsr_densify_plan.restype = _i
_lib.gsr_densify_plan.argtypes = [_i, _i, _i, _vp, _vp, _vp, _vp, _vp, ctypes.POINTER(DensifyArgs), _vp,
                                  ctypes.POINTER(_i), _vp]
_lib.gsr_densify_apply.restype = _i
_lib.gsr_densify_apply.argtypes = [_i, _i, _i, _vp, _vp, _vp, _vp, ctypes.POINTER(DensifyArgs), _vp,
                                   ctypes.POINTER(_i), _vp, _vp, _vp, _vp, _vp]

EXPORTED_SYMBOLS = ("gsr_arena_layout", "gsr_act_layout", "gsr_activate", "gsr_activation_backward",
                    "gsr_adam_step", "gsr_densify_stats", "gsr_densify_ws_bytes", "gsr_densify_plan",
                    "gsr_densify_apply", "gsr_ply_rows_to_arena", "gsr_arena_to_ply_rows", "gsr_knn_ws_bytes",
                    "gsr_dist_knn3")


class ArenaSpec:
    """Block layout of a Gaussian arena (include/gsr_train.h) for P Gaussians with M
    SH coefficients per channel and C segment classes."""

    def __init__(self, P, M, C=NUM_CLASS):
        self.P, self.M, self.C = int(P), int(M), int(C)
        off = (_ll * 7)()
        self.total = int(_lib.gsr_arena_layout(self.P, self.M, self.C, off))
        self.off = [int(o) for o in off]
        aoff = (_ll * 5)()
        self.act_total = int(_lib.gsr_act_layout(self.P, self.C, aoff))
        self.act_off = [int(o) for o in aoff]
        self.width = {"xyz": 3, "features": 3 * self.M, "opacity": 1, "scaling": 3, "rotation": 4,
                      "segment": self.C}

    def block(self, arena, name):
        """[P, width] view of one block of a parameter / gradient / moment arena."""
        b = BLOCK_NAMES.index(name)
        k = self.width[name]
        v = arena.narrow(0, self.off[b], k * self.P).view(self.P, k)
        return v.view(self.P, self.M, 3) if name == "features" else v

    def act_block(self, act, name):
        b = ("opacity", "scaling", "rotation", "segment").index(name)
        k = self.width[name]
        return act.narrow(0, self.act_off[b], k * self.P).view(self.P, k)

    def group(self, arena, gname):
        """View of one reference param group inside an arena, in the reference's shape
        (_features_dc [P,1,3], _features_rest [P,M-1,3], others [P,k])."""
        if gname == "f_dc":
            return self.block(arena, "features")[:, :1, :]
        if gname == "f_rest":
            return self.block(arena, "features")[:, 1:, :]
        return self.block(arena, gname)


def activate(spec, param, act):
    if spec.P == 0:
        return
    _check(_lib.gsr_activate(spec.P, spec.M, spec.C, param.data_ptr(), act.data_ptr(), _stream(param.device)))


def activation_backward(spec, param, act, grad):
    if spec.P == 0:
        return
    _check(_lib.gsr_activation_backward(spec.P, spec.M, spec.C, param.data_ptr(), act.data_ptr(), grad.data_ptr(),
                                        _stream(param.device)))


def adam_step(spec, param, grad, exp_avg, exp_avg_sq, act, hyper):
    if spec.P == 0:
        return
    _check(_lib.gsr_adam_step(spec.P, spec.M, spec.C, param.data_ptr(), grad.data_ptr(), exp_avg.data_ptr(),
                              exp_avg_sq.data_ptr(), act.data_ptr() if act is not None else None,
                              ctypes.byref(hyper), _stream(param.device)))


def densify_stats(dmeans2D, grad_accum, denom, update_filter=None, radii=None, max_radii2D=None):
    """gsr_densify_stats: accumulate |dmeans2D[:, :2]| and counts for the Gaussians
    selected by update_filter (bool [P]) or, if it is None, by radii > 0; also
    max_radii2D = max(max_radii2D, radii) when both are given."""
    P = int(grad_accum.numel())
    if P == 0:
        return
    dev = grad_accum.device
    checks = [(dmeans2D, "dmeans2D", torch.float32, 3 * P), (grad_accum, "xyz_gradient_accum", torch.float32, P),
              (denom, "denom", torch.float32, P)]
    if update_filter is not None:
        checks.append((update_filter, "update_filter", torch.bool, P))
    if radii is not None:
        checks.append((radii, "radii", torch.int32, P))
    if max_radii2D is not None:
        checks.append((max_radii2D, "max_radii2D", torch.float32, P))
    for t, n, dt, numel in checks:
        if t.dtype != dt or not t.is_contiguous() or t.device != dev or t.numel() != numel:
            raise RuntimeError(f"densify_stats: {n} must be a contiguous {dt} tensor of {numel} elements on {dev}")
    if update_filter is None and radii is None:
        raise RuntimeError("densify_stats: need update_filter or radii")
    ptr = lambda t: None if t is None else t.data_ptr()
    _check(_lib.gsr_densify_stats(P, ptr(update_filter), ptr(radii), dmeans2D.data_ptr(), ptr(max_radii2D),
                                  grad_accum.data_ptr(), denom.data_ptr(), _stream(dev)))


def densify(spec, param, act, exp_avg, exp_avg_sq, args, grad_accum=None, denom=None, mask=None, normals_fn=None):
    """gsr_densify_plan + gsr_densify_apply.  normals_fn(n) returns the [n, 3]
    standard-normal draws for the split children (called between the two, after
    the host learns how many are needed).  Returns (new P, new param, new exp_avg,
    new exp_avg_sq, counts)."""
    P = spec.P
    dev = param.device
    ws = torch.empty(max(1, int(_lib.gsr_densify_ws_bytes(P))), dtype=torch.uint8, device=dev)
    counts = (_i * 4)()
    ptr = lambda t: None if t is None else t.data_ptr()
    _check(_lib.gsr_densify_plan(P, spec.M, spec.C, param.data_ptr(), act.data_ptr(), ptr(grad_accum), ptr(denom),
                                 ptr(mask), ctypes.byref(args), ws.data_ptr(), counts, _stream(dev)))
    c = [int(x) for x in counts]
    n_new = c[0] + c[1] + args.split_n * c[2]
    normals = None
    if c[3] > 0 and normals_fn is not None:
        normals = normals_fn(args.split_n * c[3])
        if normals.shape != (args.split_n * c[3], 3) or normals.dtype != torch.float32 or \
                not normals.is_contiguous() or normals.device != dev:
            raise RuntimeError("densify: normals must be a contiguous float32 [split_n * n_split, 3] device tensor")
    elif c[2] > 0:
        raise RuntimeError("densify: split children need normal draws")
    new = ArenaSpec(n_new, spec.M, spec.C)
    f32 = dict(dtype=torch.float32, device=dev)
    np_, m1, m2 = (torch.empty(new.total, **f32) for _ in range(3))
    if new.total:  # padding and any block tail are defined (zero) for the float4 kernels
        for t in (np_, m1, m2):
            t.zero_()
    _check(_lib.gsr_densify_apply(P, spec.M, spec.C, param.data_ptr(), act.data_ptr(), exp_avg.data_ptr(),
                                  exp_avg_sq.data_ptr(), ctypes.byref(args), ws.data_ptr(), counts, ptr(normals),
                                  np_.data_ptr(), m1.data_ptr(), m2.data_ptr(), _stream(dev)))
    return new, np_, m1, m2, c
