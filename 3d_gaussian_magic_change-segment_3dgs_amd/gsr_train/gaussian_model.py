"""GaussianModel: the reference's Gaussian parameter container
(scene/gaussian_model.py:25-526) on one device-resident arena.

The method and attribute names are the reference's (get_xyz, get_features,
get_opacity, get_scaling, get_rotation, get_segment, training_setup,
update_learning_rate, add_densification_stats, densify_and_prune,
reset_opacity, capture / restore, save_ply / load_ply, create_from_pcd, and the
raw _xyz, _features_dc, ... tensors), so gaussian_renderer.render() and the
train.py loop drive it unchanged.  What differs is the storage:

* one fp32 parameter arena (include/gsr_train.h) is the single nn.Parameter;
  the reference's seven tensors are views of it;
* the activations are one HIP pass (gsr_activate) -- or none at all, because
  GaussianAdam.step() writes them while it updates the parameters -- instead of
  a dozen torch kernels plus a torch.cat of the SH features;
* the rasterizer's gradient arena has the same block layout, so the activation
  backward runs in place on it and it becomes the arena's .grad without a copy;
* the optimizer is GaussianAdam (one fused launch for all seven groups).

Editing the raw views in place (e.g. `model._opacity.fill_(0)`) is allowed;
call `model.invalidate()` afterwards so the activated copy is refreshed.
"""
import os

import numpy as np
import torch
import torch.nn as nn

from . import _C
from . import ply as _ply
from .optim import GaussianAdam


def inverse_sigmoid(x):
    """utils/general_utils.py:18-19."""
    return torch.log(x / (1 - x))


def get_expon_lr_func(lr_init, lr_final, lr_delay_steps=0, lr_delay_mult=1.0, max_steps=1000000):
    """Log-linear learning-rate decay with an optional sine warm-up of the delay
    factor; restates utils/general_utils.py:37-70 (numpy float64)."""

    def helper(step):
        if step < 0 or (lr_init == 0.0 and lr_final == 0.0):
            return 0.0
        if lr_delay_steps > 0:
            ramp = np.clip(step / lr_delay_steps, 0, 1)
            delay_rate = lr_delay_mult + (1 - lr_delay_mult) * np.sin(0.5 * np.pi * ramp)
        else:
            delay_rate = 1.0
        t = np.clip(step / max_steps, 0, 1)
        return delay_rate * np.exp(np.log(lr_init) * (1 - t) + np.log(lr_final) * t)

    return helper


# How the activation backward got its gradient arena (tests check the zero-copy path).
BACKWARD_PATHS = {"zero_copy": 0, "packed": 0}


class _Activations(torch.autograd.Function):
    """Raw arena -> (xyz, features, opacity, scaling, rotation, segment) as consumed
    by the rasterizer.  xyz and features are views of the arena; the other four
    are views of the activated buffer (filled by gsr_activate or the last Adam
    step).  Backward: one in-place gsr_activation_backward on the gradient arena."""

    @staticmethod
    def forward(ctx, arena, act, spec):
        ctx.spec, ctx.param, ctx.act = spec, arena.detach(), act
        return (spec.block(arena, "xyz"), spec.block(arena, "features"), spec.act_block(act, "opacity"),
                spec.act_block(act, "scaling"), spec.act_block(act, "rotation"), spec.act_block(act, "segment"))

    @staticmethod
    def backward(ctx, *grads):
        spec = ctx.spec
        g = _shared_grad_arena(spec, grads)
        BACKWARD_PATHS["packed" if g is None else "zero_copy"] += 1
        if g is None:  # gradients not all from one rasterizer call: pack them
            g = torch.zeros(spec.total, dtype=torch.float32, device=ctx.param.device)
            for b, t in enumerate(grads):
                if t is not None:
                    n = spec.width[_C.BLOCK_NAMES[b]] * spec.P
                    g.narrow(0, spec.off[b], n).copy_(t.reshape(-1))
        _C.activation_backward(spec, ctx.param, ctx.act, g)
        return g, None, None


def _shared_grad_arena(spec, grads):
    """If the six incoming gradients are the blocks of one rasterizer gradient
    arena (diff_gaussian_rasterization._C.grad_arena_layout), return that arena's
    first spec.total floats (a view: no copy)."""
    if any(t is None for t in grads):
        return None
    base = grads[0]._base
    if base is None or base.dtype != torch.float32 or base.dim() != 1 or not base.is_contiguous():
        return None
    if base.numel() < spec.total:
        return None
    p0 = base.data_ptr()
    for b, t in enumerate(grads):
        if t._base is not base or not t.is_contiguous() or t.data_ptr() != p0 + 4 * spec.off[b]:
            return None
    return base.narrow(0, 0, spec.total)


class GaussianModel:
    def __init__(self, sh_degree: int, num_class=2, device="cuda"):
        self.active_sh_degree = 0
        self.max_sh_degree = int(sh_degree)
        self.num_class = int(num_class)
        self.device = torch.device(device)
        self.optimizer = None
        self.percent_dense = 0
        self.spatial_lr_scale = 0
        self._allocate(0)

    # ---- storage ------------------------------------------------------------------------
    @property
    def _M(self):
        return (self.max_sh_degree + 1) ** 2

    def _allocate(self, P):
        self._spec = _C.ArenaSpec(P, self._M, self.num_class)
        f32 = dict(dtype=torch.float32, device=self.device)
        self._arena = nn.Parameter(torch.zeros(self._spec.total, **f32))
        self._act = torch.zeros(self._spec.act_total, **f32)
        self.max_radii2D = torch.zeros(P, **f32)
        self.xyz_gradient_accum = torch.zeros((P, 1), **f32)
        self.denom = torch.zeros((P, 1), **f32)
        self._params_changed()

    def _params_changed(self, act_fresh=False):
        self._cache = {}
        self._act_fresh = act_fresh

    def invalidate(self):
        """Raw parameters were edited in place: recompute the activations on next use."""
        self._params_changed(act_fresh=False)

    def group_view(self, name):
        """Detached view of one reference parameter tensor inside the arena."""
        return self._spec.group(self._arena.data, name)

    _xyz = property(lambda self: self.group_view("xyz"))
    _features_dc = property(lambda self: self.group_view("f_dc"))
    _features_rest = property(lambda self: self.group_view("f_rest"))
    _opacity = property(lambda self: self.group_view("opacity"))
    _segment = property(lambda self: self.group_view("segment"))
    _scaling = property(lambda self: self.group_view("scaling"))
    _rotation = property(lambda self: self.group_view("rotation"))

    @property
    def num_points(self):
        return self._spec.P

    def _activations(self):
        mode = torch.is_grad_enabled()
        hit = self._cache.get(mode)
        if hit is not None:
            return hit
        if not self._act_fresh:
            _C.activate(self._spec, self._arena.data, self._act)
            self._act_fresh = True
        if mode:
            outs = _Activations.apply(self._arena, self._act, self._spec)
        else:
            s, a, act = self._spec, self._arena.data, self._act
            outs = (s.block(a, "xyz"), s.block(a, "features"), s.act_block(act, "opacity"),
                    s.act_block(act, "scaling"), s.act_block(act, "rotation"), s.act_block(act, "segment"))
        self._cache[mode] = outs
        return outs

    # ---- reference accessors (gaussian_model.py:100-127) ---------------------------------
    get_xyz = property(lambda self: self._activations()[0])
    get_features = property(lambda self: self._activations()[1])
    get_opacity = property(lambda self: self._activations()[2])
    get_scaling = property(lambda self: self._activations()[3])
    get_rotation = property(lambda self: self._activations()[4])
    get_segment = property(lambda self: self._activations()[5])

    def get_covariance(self, scaling_modifier=1):
        """build_covariance_from_scaling_rotation (gaussian_model.py:28-32): upper
        triangle of (R S)(R S)^T with R from the raw quaternion."""
        s = self.get_scaling * scaling_modifier
        R = build_rotation(self._rotation)
        L = R * s[:, None, :]
        cov = L @ L.transpose(1, 2)
        idx = torch.tensor([[0, 0], [0, 1], [0, 2], [1, 1], [1, 2], [2, 2]], device=cov.device)
        return cov[:, idx[:, 0], idx[:, 1]]

    def oneupSHdegree(self):
        if self.active_sh_degree < self.max_sh_degree:
            self.active_sh_degree += 1

    # ---- construction ----------------------------------------------------------------------
    @torch.no_grad()
    def create_from_tensors(self, xyz, features_dc, features_rest, opacity, segment, scaling, rotation):
        """Fill the arena from raw (pre-activation) tensors in the reference's shapes:
        xyz [P,3], features_dc [P,1,3], features_rest [P,M-1,3], opacity [P,1],
        segment [P,C], scaling [P,3] (log), rotation [P,4] (wxyz, unnormalised)."""
        P = int(xyz.shape[0])
        self._allocate(P)
        for name, t in (("xyz", xyz), ("f_dc", features_dc), ("f_rest", features_rest), ("opacity", opacity),
                        ("segment", segment), ("scaling", scaling), ("rotation", rotation)):
            v = self.group_view(name)
            t = torch.as_tensor(t, dtype=torch.float32)
            if t.numel() != v.numel():
                raise ValueError(f"create_from_tensors: {name} has {t.numel()} values, expected {tuple(v.shape)}")
            v.copy_(t.reshape(v.shape).to(self.device))
        self._params_changed()
        return self

    @torch.no_grad()
    def create_from_pcd(self, pcd, spatial_lr_scale: float):
        """gaussian_model.py:129-156: SH DC from the point colours (RGB2SH), scales
        from the 3-NN mean squared distance (distCUDA2 -> csrc/knn.hip), identity
        rotations, opacity and segment logits of 0.1."""
        from .knn import distCUDA2
        self.spatial_lr_scale = spatial_lr_scale
        pts = torch.as_tensor(np.asarray(pcd.points), dtype=torch.float32).to(self.device)
        cols = torch.as_tensor(np.asarray(pcd.colors), dtype=torch.float32).to(self.device)
        P, M = pts.shape[0], self._M
        f_dc = ((cols - 0.5) / 0.28209479177387814).reshape(P, 1, 3)  # RGB2SH (utils/sh_utils.py:114-115)
        f_rest = torch.zeros((P, M - 1, 3), dtype=torch.float32, device=self.device)
        dist2 = torch.clamp_min(distCUDA2(pts), 0.0000001)
        scales = torch.log(torch.sqrt(dist2))[..., None].repeat(1, 3)
        rots = torch.zeros((P, 4), dtype=torch.float32, device=self.device)
        rots[:, 0] = 1
        opac = inverse_sigmoid(0.1 * torch.ones((P, 1), dtype=torch.float32, device=self.device))
        segs = inverse_sigmoid(0.1 * torch.ones((P, self.num_class), dtype=torch.float32, device=self.device))
        self.create_from_tensors(pts, f_dc, f_rest, opac, segs, scales, rots)

    def training_setup(self, training_args):
        """gaussian_model.py:158-177 with GaussianAdam in place of torch.optim.Adam."""
        self.percent_dense = training_args.percent_dense
        P = self.num_points
        self.xyz_gradient_accum = torch.zeros((P, 1), dtype=torch.float32, device=self.device)
        self.denom = torch.zeros((P, 1), dtype=torch.float32, device=self.device)
        ta = training_args
        groups = [
            {"params": [self._xyz], "lr": ta.position_lr_init * self.spatial_lr_scale, "name": "xyz"},
            {"params": [self._features_dc], "lr": ta.feature_lr, "name": "f_dc"},
            {"params": [self._features_rest], "lr": ta.feature_lr / 20.0, "name": "f_rest"},
            {"params": [self._opacity], "lr": ta.opacity_lr, "name": "opacity"},
            {"params": [self._segment], "lr": ta.segment_lr, "name": "segment"},
            {"params": [self._scaling], "lr": ta.scaling_lr, "name": "scaling"},
            {"params": [self._rotation], "lr": ta.rotation_lr, "name": "rotation"},
        ]
        self.optimizer = GaussianAdam(self, groups, lr=0.0, eps=1e-15)
        self.xyz_scheduler_args = get_expon_lr_func(lr_init=ta.position_lr_init * self.spatial_lr_scale,
                                                    lr_final=ta.position_lr_final * self.spatial_lr_scale,
                                                    lr_delay_mult=ta.position_lr_delay_mult,
                                                    max_steps=ta.position_lr_max_steps)

    def update_learning_rate(self, iteration):
        for group in self.optimizer.param_groups:
            if group["name"] == "xyz":
                lr = self.xyz_scheduler_args(iteration)
                group["lr"] = lr
                return lr

    # ---- checkpoints (gaussian_model.py:64-98) --------------------------------------------
    def capture(self):
        c = lambda n: self.group_view(n).clone()
        return (self.active_sh_degree, c("xyz"), c("f_dc"), c("f_rest"), c("scaling"), c("rotation"), c("opacity"),
                c("segment"), self.max_radii2D.clone(), self.xyz_gradient_accum.clone(), self.denom.clone(),
                self.optimizer.state_dict(), self.spatial_lr_scale)

    def restore(self, model_args, training_args):
        (self.active_sh_degree, xyz, f_dc, f_rest, scaling, rotation, opacity, segment, max_radii2D,
         xyz_gradient_accum, denom, opt_dict, self.spatial_lr_scale) = model_args
        self.create_from_tensors(xyz.detach(), f_dc.detach(), f_rest.detach(), opacity.detach(), segment.detach(),
                                 scaling.detach(), rotation.detach())
        self.training_setup(training_args)
        self.max_radii2D = max_radii2D.to(self.device, torch.float32).contiguous()
        self.xyz_gradient_accum = xyz_gradient_accum.to(self.device, torch.float32).contiguous()
        self.denom = denom.to(self.device, torch.float32).contiguous()
        self.optimizer.load_state_dict(opt_dict)

    # ---- densification statistics / opacity reset -------------------------------------
    @torch.no_grad()
    def add_densification_stats(self, viewspace_point_tensor, update_filter):
        """gaussian_model.py:523-526 as one kernel (gsr_densify_stats)."""
        grad = viewspace_point_tensor.grad if isinstance(viewspace_point_tensor, torch.Tensor) and \
            viewspace_point_tensor.grad is not None else viewspace_point_tensor
        _C.densify_stats(grad.contiguous(), self.xyz_gradient_accum, self.denom,
                         update_filter=update_filter.to(torch.bool).contiguous())

    @torch.no_grad()
    def update_densification_stats(self, viewspace_point_tensor, radii):
        """train.py:170-172 in one kernel: max_radii2D[vis] = max(max_radii2D[vis],
        radii[vis]) and add_densification_stats(viewspace, vis) with vis = radii > 0."""
        grad = viewspace_point_tensor.grad if viewspace_point_tensor.grad is not None else viewspace_point_tensor
        _C.densify_stats(grad.contiguous(), self.xyz_gradient_accum, self.denom, radii=radii.to(torch.int32),
                         max_radii2D=self.max_radii2D)

    @torch.no_grad()
    def reset_opacity(self):
        """gaussian_model.py:264-268: opacity <- inverse_sigmoid(min(sigmoid(opacity),
        0.01)); that group's Adam moments are zeroed (replace_tensor_to_optimizer)."""
        op = self.get_opacity
        new = inverse_sigmoid(torch.min(op, torch.ones_like(op) * 0.01))
        self.group_view("opacity").copy_(new)
        if self.optimizer is not None:
            self.optimizer._reset_group("opacity")
        self._params_changed()

    # ---- densification (gaussian_model.py:386-521) ---------------------------------------
    def _densify_args(self, mode, max_grad=0.0, min_opacity=0.0, extent=0.0, max_screen_size=None, N=2):
        a = _C.DensifyArgs()
        a.mode, a.split_n = mode, int(N)
        a.max_grad, a.min_opacity = float(max_grad), float(min_opacity)
        a.clone_max_scale = float(self.percent_dense * extent)
        a.prune_max_scale = float(0.1 * extent)
        a.max_screen_size = float(max_screen_size) if max_screen_size else 0.0
        a.split_divisor = float(0.8 * N)
        return a

    @torch.no_grad()
    def _rebuild(self, args, grad_accum=None, denom=None, mask=None, generator=None):
        if not self._act_fresh:
            _C.activate(self._spec, self._arena.data, self._act)
            self._act_fresh = True
        opt = self.optimizer
        m1 = opt.exp_avg if opt is not None else torch.zeros_like(self._arena.data)
        m2 = opt.exp_avg_sq if opt is not None else torch.zeros_like(self._arena.data)

        def normals(n):  # torch.normal(mean=0, std=s) draws z ~ N(0,1) as normal_ then scales
            return torch.empty((n, 3), dtype=torch.float32, device=self.device).normal_(0.0, 1.0, generator=generator)

        spec, p, m1n, m2n, counts = _C.densify(self._spec, self._arena.data, self._act, m1, m2, args,
                                               grad_accum=grad_accum, denom=denom, mask=mask, normals_fn=normals)
        self._spec = spec
        self._arena = nn.Parameter(p)
        self._act = torch.zeros(spec.act_total, dtype=torch.float32, device=self.device)
        self._params_changed()
        if opt is not None:
            opt._resize(m1n, m2n)
        P = spec.P
        # densification_postfix (:402-404) resets the statistics; prune keeps the zeros
        self.xyz_gradient_accum = torch.zeros((P, 1), dtype=torch.float32, device=self.device)
        self.denom = torch.zeros((P, 1), dtype=torch.float32, device=self.device)
        self.max_radii2D = torch.zeros(P, dtype=torch.float32, device=self.device)
        return counts

    def densify_and_prune(self, max_grad, min_opacity, extent, max_screen_size, generator=None):
        """gaussian_model.py:508-521: clone, split (N = 2) and prune in one plan +
        apply pair of kernels; new Gaussians get zero Adam moments."""
        a = self._densify_args(_C.DENSIFY_AND_PRUNE, max_grad, min_opacity, extent, max_screen_size)
        return self._rebuild(a, self.xyz_gradient_accum.contiguous(), self.denom.contiguous(), generator=generator)

    def densify_and_clone(self, grads, grad_threshold, scene_extent):
        """gaussian_model.py:439-457 (grads: [P, 1] mean view-space gradients)."""
        a = self._densify_args(_C.CLONE_ONLY, grad_threshold, 0.0, scene_extent)
        g = grads.reshape(-1).to(self.device, torch.float32).contiguous()
        return self._rebuild(a, g, torch.ones_like(g))

    def densify_and_split(self, grads, grad_threshold, scene_extent, N=2, generator=None):
        """gaussian_model.py:406-437 (selected originals are removed, N children each)."""
        a = self._densify_args(_C.SPLIT_ONLY, grad_threshold, 0.0, scene_extent, N=N)
        P = self.num_points
        g = torch.zeros(P, dtype=torch.float32, device=self.device)
        src = grads.reshape(-1).to(self.device, torch.float32)
        g[:src.numel()] = src  # padded_grad
        return self._rebuild(a, g, torch.ones_like(g), generator=generator)

    def prune_points(self, mask):
        """gaussian_model.py:340-357: drop mask[i] (bool [P]); moments and statistics
        follow the kept Gaussians (statistics are kept, not reset, like the reference)."""
        keep_stats = (self.xyz_gradient_accum, self.denom, self.max_radii2D)
        a = self._densify_args(_C.PRUNE_MASK)
        m = mask.reshape(-1).to(self.device, torch.bool).contiguous()
        counts = self._rebuild(a, mask=m)
        keep = ~m
        self.xyz_gradient_accum = keep_stats[0][keep].contiguous()
        self.denom = keep_stats[1][keep].contiguous()
        self.max_radii2D = keep_stats[2][keep].contiguous()
        return counts

    def construct_list_of_attributes(self):
        """gaussian_model.py:187-205: PLY vertex property names in file order."""
        return _ply.attribute_names(self._M, self.num_class)

    # ---- PLY (gaussian_model.py:207-338; merge: visualizer.py:196-226) ---------------------
    @torch.no_grad()
    def save_ply(self, path, mask=None):
        """Binary little-endian PLY of the raw parameters, attribute order of
        construct_list_of_attributes (normals written as 0).  The arena -> row
        transposition runs on the GPU; one D2H copy of the vertex block."""
        d = os.path.dirname(path)
        if d:
            os.makedirs(d, exist_ok=True)
        names = self.construct_list_of_attributes()
        rows = _ply.arena_to_rows(self._spec, self._arena.data, names)
        if mask is not None:
            rows = rows[mask.to(rows.device)]
        _ply.write_rows(path, names, rows.cpu().numpy())

    def save_ply_using_mask(self, path, mask):
        """gaussian_model.py:226-262 (every attribute masked, segments included)."""
        self.save_ply(path, mask=mask)

    @torch.no_grad()
    def load_ply(self, path):
        """gaussian_model.py:270-315: one H2D copy of the vertex block, transposed
        into the arena on the GPU; active_sh_degree = max_sh_degree."""
        self.merge_ply([path])
        self.active_sh_degree = self.max_sh_degree

    @torch.no_grad()
    def merge_ply(self, paths):
        """Load several PLY scenes into one model, concatenated in order (the
        reference's _merge_scenes, visualizer.py:196-226).  Returns
        ([(start_offset, end_offset)] per scene, point_object_id int32 [P])."""
        files = [_ply.read_rows(p) for p in paths]
        P = sum(r.shape[0] for _, r in files)
        self._allocate(P)
        offsets, o = [], 0
        for names, rows in files:
            _ply.arena_columns(names, self._M, self.num_class)  # validate before any upload
        for names, rows in files:
            n = rows.shape[0]
            if n:
                dev_rows = torch.from_numpy(rows).pin_memory().to(self.device, non_blocking=True)
                _ply.rows_to_arena(self._spec, self._arena.data, dev_rows, names, dst=o)
            offsets.append((o, o + n))
            o += n
        ids = torch.zeros(P, dtype=torch.int32, device=self.device)
        for k, (a, b) in enumerate(offsets):
            ids[a:b] = k
        self._params_changed()
        self.active_sh_degree = self.max_sh_degree
        return offsets, ids

    def load_ply_no_instance(self, path):
        """gaussian_model.py:317-352: host arrays (xyz, features_dc [P,3,1],
        features_extra [P,3,M-1], opacities, scales, rots, segments)."""
        names, rows = _ply.read_rows(path)
        col = _ply.arena_columns(names, self._M, self.num_class)
        M, C = self._M, self.num_class
        take = lambda ks: rows[:, [col[k] for k in ks]].astype(np.float64)
        xyz = take(range(3))
        feats = take(range(3, 3 + 3 * M)).reshape(-1, M, 3)  # [P, M, 3]
        o = 3 + 3 * M
        opac = take([o])
        scales = take(range(o + 1, o + 4))
        rots = take(range(o + 4, o + 8))
        segs = take(range(o + 8, o + 8 + C))
        return (xyz, feats[:, :1].transpose(0, 2, 1), feats[:, 1:].transpose(0, 2, 1), opac, scales, rots, segs)

    def instance_parm(self, xyz, features_dc, features_extra, opacities, scales, rots, segments):
        """gaussian_model.py:354-367 (features_dc [P,3,1], features_extra [P,3,M-1])."""
        t = lambda a: torch.as_tensor(np.asarray(a), dtype=torch.float32)
        self.create_from_tensors(t(xyz), t(features_dc).transpose(1, 2), t(features_extra).transpose(1, 2),
                                 t(opacities), t(segments), t(scales), t(rots))
        self.active_sh_degree = self.max_sh_degree


def build_rotation(r):
    """utils/general_utils.py:86-107: rotation matrices of the normalised quaternions (wxyz)."""
    q = r / torch.sqrt((r * r).sum(dim=1))[:, None]
    w, x, y, z = q.unbind(1)
    return torch.stack([
        1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y),
        2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x),
        2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y),
    ], dim=1).view(-1, 3, 3)
