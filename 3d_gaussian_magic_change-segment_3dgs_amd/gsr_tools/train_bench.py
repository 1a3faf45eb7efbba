"""Measurement of the training step around the rasterizer,
reported by bench.py under "train_step".

Fused path (gsr_train): GaussianModel arena + GaussianAdam -- one gsr_adam_step
launch per iteration (it also writes the activations the next render reads) and
one in-place gsr_activation_backward on the rasterizer's gradient arena.
Reference path: the same work the reference's way (scene/gaussian_model.py,
train.py:183-185) -- seven nn.Parameters, torch activations + torch.cat of the SH
features, autograd backward of those, torch.optim.Adam(eps=1e-15) over seven
param groups -- timed on the same GPU, with the same rasterizer in between.
"""
import torch

HBM_PEAK_GBS = 8000.0


def adam_bytes(P, M, C=2):
    """Algorithmic HBM bytes of one fused Adam step: read param, grad, exp_avg,
    exp_avg_sq and write param, exp_avg, exp_avg_sq for every float of the
    Gaussian (3 + 3M + 1 + 3 + 4 + C floats), plus the activated opacity /
    scaling / rotation / segment written for the next forward."""
    F = 3 + 3 * M + 1 + 3 + 4 + C
    return P * (28 * F + 4 * (1 + 3 + 4 + C))


def act_bwd_bytes(P, C=2):
    """In-place activation backward: read grad + (act or raw) and write grad for the
    opacity / scaling / rotation / segment blocks."""
    return P * 12 * (1 + 3 + 4 + C)


_SPREAD = {}


def _events_ms(fn, reps, repeats=5):
    """Median over `repeats` timings of `reps` back-to-back calls (ms per call); the
    min / max of the repeats are kept in _SPREAD[fn] for the report."""
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(repeats):
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) / reps)
    ts.sort()
    _SPREAD[fn] = (ts[0], ts[-1])
    return ts[len(ts) // 2]


def _spread(fn):
    lo, hi = _SPREAD.get(fn, (None, None))
    return {"min": round(lo, 4), "max": round(hi, 4), "repeats": 5} if lo is not None else None


class _TrainArgs:
    position_lr_init, position_lr_final, position_lr_delay_mult, position_lr_max_steps = 1.6e-4, 1.6e-6, 0.01, 30000
    feature_lr, opacity_lr, segment_lr, scaling_lr, rotation_lr, percent_dense = 0.0025, 0.05, 0.05, 0.005, 0.001, 0.01


def measure(scene_cpu, cam_cpu, ups, device, reps=20, iters=10):
    from gsr_train import GaussianModel
    import diff_gaussian_rasterization as dgr

    P, deg = scene_cpu.P, scene_cpu.sh_degree
    M = (deg + 1) ** 2
    raw = {"xyz": scene_cpu.means3D, "f_dc": scene_cpu.shs[:, :1], "f_rest": scene_cpu.shs[:, 1:],
           "opacity": torch.logit(scene_cpu.opacities), "segment": torch.logit(scene_cpu.segments),
           "scaling": torch.log(scene_cpu.scales), "rotation": scene_cpu.rotations}
    m = GaussianModel(deg, device=device)
    m.create_from_tensors(*(raw[k] for k in ("xyz", "f_dc", "f_rest", "opacity", "segment", "scaling", "rotation")))
    m.spatial_lr_scale = 1.0
    m.training_setup(_TrainArgs)
    m.active_sh_degree = deg
    gen = torch.Generator(device=device).manual_seed(3)
    g_arena = torch.randn(m._spec.total, device=device, generator=gen) * 1e-3

    def fused_adam():
        m._arena.grad = g_arena
        m.optimizer.step()

    adam_ms = _events_ms(fused_adam, reps)
    from gsr_train import _C as T
    g_work = g_arena.clone()
    actbwd_ms = _events_ms(lambda: T.activation_backward(m._spec, m._arena.data, m._act, g_work), reps)
    m.optimizer.zero_grad()

    # reference style: seven parameters, torch activations, torch.optim.Adam
    params = {k: torch.nn.Parameter(v.detach().to(device).contiguous().clone()) for k, v in raw.items()}
    groups = [{"params": [params["xyz"]], "lr": 1.6e-4, "name": "xyz"},
              {"params": [params["f_dc"]], "lr": 0.0025, "name": "f_dc"},
              {"params": [params["f_rest"]], "lr": 0.0025 / 20, "name": "f_rest"},
              {"params": [params["opacity"]], "lr": 0.05, "name": "opacity"},
              {"params": [params["segment"]], "lr": 0.05, "name": "segment"},
              {"params": [params["scaling"]], "lr": 0.005, "name": "scaling"},
              {"params": [params["rotation"]], "lr": 0.001, "name": "rotation"}]
    opt = torch.optim.Adam(groups, lr=0.0, eps=1e-15)
    for k, p in params.items():
        p.grad = torch.randn(p.shape, device=device, generator=gen) * 1e-3
    ref_adam_ms = _events_ms(opt.step, reps)

    def ref_acts():
        return (params["xyz"], torch.cat((params["f_dc"], params["f_rest"]), dim=1), torch.sigmoid(params["opacity"]),
                torch.exp(params["scaling"]), torch.nn.functional.normalize(params["rotation"]),
                torch.sigmoid(params["segment"]))

    act_grads = [torch.randn(t.shape, device=device, generator=gen) * 1e-3 for t in ref_acts()]

    def ref_act_fwd_bwd():
        torch.autograd.backward(list(ref_acts()), act_grads)

    ref_act_ms = _events_ms(ref_act_fwd_bwd, reps)

    # whole training iteration: activations -> rasterizer fwd+bwd -> activation bwd -> Adam
    st = dgr.GaussianRasterizationSettings(
        image_height=cam_cpu.height, image_width=cam_cpu.width, tanfovx=cam_cpu.tanfovx, tanfovy=cam_cpu.tanfovy,
        bg=torch.zeros(3, device=device), scale_modifier=1.0, viewmatrix=cam_cpu.world_view_transform.to(device),
        projmatrix=cam_cpu.full_proj_transform.to(device), sh_degree=deg, campos=cam_cpu.camera_center.to(device),
        prefiltered=False, debug=False)
    rast = dgr.GaussianRasterizer(st)
    up = [ups["color"], ups["depth"], ups["alpha"], ups["segment"]]

    def render_backward(xyz, feats, op, sc, rot, seg):
        means2D = torch.zeros_like(xyz, requires_grad=True)
        color, radii, depth, alpha, segment = rast(means3D=xyz, means2D=means2D, shs=feats, colors_precomp=None,
                                                   segments=seg, opacities=op, scales=sc, rotations=rot,
                                                   cov3D_precomp=None)
        torch.autograd.backward([color, depth, alpha, segment], up)

    def fused_iter():
        render_backward(m.get_xyz, m.get_features, m.get_opacity, m.get_scaling, m.get_rotation, m.get_segment)
        m.optimizer.step()
        m.optimizer.zero_grad(set_to_none=True)

    def ref_iter():
        render_backward(*ref_acts())
        opt.step()
        opt.zero_grad(set_to_none=True)

    fused_iter_ms = _events_ms(fused_iter, iters)
    ref_iter_ms = _events_ms(ref_iter, iters)

    # densify_and_prune once on the trained model (statistics: mean grad ~U[0, 4e-4])
    P0 = m.num_points
    m.xyz_gradient_accum.uniform_(0.0, 4e-4, generator=gen)
    m.denom.fill_(1.0)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    counts = m.densify_and_prune(2e-4, 0.005, 1.5, 20, generator=gen)
    b.record()
    b.synchronize()
    densify_ms = a.elapsed_time(b)

    # distCUDA2 (create_from_pcd) on the scene's means
    from gsr_train import distCUDA2
    pts = scene_cpu.means3D.to(device)
    knn_ms = _events_ms(lambda: distCUDA2(pts), 3, repeats=3)
    ab = adam_bytes(P, M)
    return {
        "workload": f"P={P}, SH{deg}, 7 param groups (scene/gaussian_model.py:162-170)",
        "timing": "median of 5 repeats of back-to-back calls (hipEvents)",
        "adam_step": {"ms": round(adam_ms, 4), "spread_ms": _spread(fused_adam), "algorithmic_bytes": ab,
                      "achieved_gbs": round(ab / (adam_ms * 1e-3) / 1e9, 1),
                      "frac": round(ab / (adam_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4), "bound": "hbm"},
        "activation_backward": {"ms": round(actbwd_ms, 4),
                                "achieved_gbs": round(act_bwd_bytes(P) / (actbwd_ms * 1e-3) / 1e9, 1)},
        "reference_torch": {"adam_ms": round(ref_adam_ms, 4), "activations_fwd_bwd_ms": round(ref_act_ms, 4),
                            "note": "torch.optim.Adam (default foreach) + torch activations/cat and their "
                                    "autograd backward, same GPU"},
        "train_iteration_ms": {"fused": round(fused_iter_ms, 4), "reference_style": round(ref_iter_ms, 4),
                               "fused_spread": _spread(fused_iter),
                               "note": "activations + rasterizer fwd+bwd (this library) + activation bwd + "
                                       "Adam step, one view"},
        "densify_and_prune": {"ms": round(densify_ms, 3), "P_before": P0, "P_after": m.num_points,
                              "counts": counts, "note": "plan (classify + 4 scans) + host sync + apply"},
        "dist_knn3": {"ms": round(knn_ms, 3), "P": P},
    }
