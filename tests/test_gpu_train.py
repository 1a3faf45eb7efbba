"""Training step around the rasterizer on the GPU:
activations, activation backward (both the zero-copy rasterizer path and the
packed path), the fused Adam step and the densification statistics, against the
CPU oracle oracle/train_oracle.py (torch CPU ops + torch.optim.Adam, i.e. the
reference's own arithmetic).

Tolerances (fp32): activations and their backward agree to a few ulp (exp /
sigmoid / sqrt are libm-accurate on both sides, not bit-identical), so
rtol 2e-6 / atol 1e-7 relative to the value scale (the normalize
backward cancels its radial component, so its tolerance is relative to the size
of its terms, rot_atol); Adam parameters after several
steps rtol 1e-5 / atol 1e-6 (the update is lr * m / sqrt(v) -- a ratio of
rounded moments); densification statistics rtol 1e-6, counts exact.
"""
import numpy as np
import pytest
import torch

import harness as Hn
from gsr_tools.scene import synthetic_scene, orbit_camera
from oracle.train_oracle import RefGaussians, GROUPS

pytestmark = pytest.mark.gpu

DEV = "cuda"


def raw_params(P, sh_degree=3, seed=0):
    """Raw (pre-activation) parameters of a synthetic scene, reference shapes."""
    sc = synthetic_scene(P, sh_degree=sh_degree, seed=seed)
    g = torch.Generator().manual_seed(seed + 100)
    rot = sc.rotations * (0.5 + torch.rand(P, 1, generator=g) * 2.0)  # unnormalised quaternions
    rot[:3] = torch.tensor([[1e-14, 0, 0, 0], [0, 0, 0, 0], [3.0, -4.0, 0.0, 12.0]])  # eps clamp + exact norms
    return {"xyz": sc.means3D, "f_dc": sc.shs[:, :1].contiguous(), "f_rest": sc.shs[:, 1:].contiguous(),
            "opacity": torch.logit(sc.opacities), "segment": torch.logit(sc.segments),
            "scaling": torch.log(sc.scales), "rotation": rot.contiguous()}


def make_model(raw, sh_degree=3):
    from gsr_train import GaussianModel
    m = GaussianModel(sh_degree, device=DEV)
    m.create_from_tensors(raw["xyz"], raw["f_dc"], raw["f_rest"], raw["opacity"], raw["segment"], raw["scaling"],
                          raw["rotation"])
    return m


def make_ref(raw):
    return RefGaussians(raw["xyz"], raw["f_dc"], raw["f_rest"], raw["opacity"], raw["segment"], raw["scaling"],
                        raw["rotation"])


def rot_atol(g_act_rot, raw_rot, rel=4e-6):
    """Absolute tolerance per row for d(raw rotation): the normalize backward
    g/d - x (x.g)/d^3 cancels its radial part, so rounding is relative to the
    size of the terms, |g|/d, not to the (possibly much smaller) result."""
    g = torch.as_tensor(g_act_rot).float().cpu()
    d = torch.as_tensor(raw_rot).float().cpu().norm(dim=1).clamp_min(1e-12)
    return (rel * g.abs().max(dim=1).values / d)[:, None].numpy()


def close(a, b, rtol, atol, what):
    a = a.detach().float().cpu().numpy() if torch.is_tensor(a) else np.asarray(a)
    b = b.detach().float().cpu().numpy() if torch.is_tensor(b) else np.asarray(b)
    assert a.shape == b.shape, f"{what}: shape {a.shape} vs {b.shape}"
    err = np.abs(a - b)
    bad = err > atol + rtol * np.abs(b)
    assert not bad.any(), f"{what}: {bad.sum()} mismatches, max err {err.max():.3e} at {np.argmax(err)}"


LR = {"xyz": 1.6e-4, "f_dc": 0.0025, "f_rest": 0.0025 / 20, "opacity": 0.05, "segment": 0.05, "scaling": 0.005,
      "rotation": 0.001}


class _Args:
    position_lr_init, position_lr_final, position_lr_delay_mult, position_lr_max_steps = 1.6e-4, 1.6e-6, 0.01, 30000
    feature_lr, opacity_lr, segment_lr, scaling_lr, rotation_lr, percent_dense = 0.0025, 0.05, 0.05, 0.005, 0.001, 0.01


def test_activations_match_reference(gpu_available):
    raw = raw_params(5003)
    m, ref = make_model(raw), make_ref(raw)
    with torch.no_grad():
        a = ref.activated()
        close(m.get_xyz, a["xyz"], 0, 0, "xyz")
        close(m.get_features, a["features"], 0, 0, "features")
        close(m.get_opacity, a["opacity"], 2e-6, 1e-7, "opacity")
        close(m.get_segment, a["segment"], 2e-6, 1e-7, "segment")
        close(m.get_scaling, a["scaling"], 2e-6, 1e-12, "scaling")
        close(m.get_rotation, a["rotation"], 2e-6, 1e-7, "rotation")
        # the raw reference tensors are views of the arena
        close(m._features_rest, raw["f_rest"], 0, 0, "_features_rest")
        close(m._rotation, raw["rotation"], 0, 0, "_rotation")


def test_activation_backward_packed(gpu_available):
    """Gradients arriving from ordinary torch ops (not one rasterizer arena)."""
    from gsr_train import gaussian_model as GM
    raw = raw_params(4097)
    m, ref = make_model(raw), make_ref(raw)
    g = torch.Generator().manual_seed(7)
    grads = {k: torch.randn(v.shape, generator=g) for k, v in ref.activated().items()}
    before = dict(GM.BACKWARD_PATHS)
    outs = [m.get_xyz, m.get_features, m.get_opacity, m.get_scaling, m.get_rotation, m.get_segment]
    keys = ["xyz", "features", "opacity", "scaling", "rotation", "segment"]
    torch.autograd.backward(outs, [grads[k].to(DEV) for k in keys])
    assert GM.BACKWARD_PATHS["packed"] == before["packed"] + 1
    ref.backward_from_activated(grads)
    for name in GROUPS:
        close(m._spec.group(m._arena.grad, name), ref.params[name].grad, 5e-6,
              rot_atol(grads["rotation"], raw["rotation"]) if name == "rotation" else 1e-7, f"d{name}")


def test_activation_backward_zero_copy_through_rasterizer(gpu_available):
    """render() style call: the model's activated tensors into GaussianRasterizer;
    the rasterizer's gradient arena becomes the arena .grad in place."""
    from diff_gaussian_rasterization import GaussianRasterizer
    from gsr_train import gaussian_model as GM
    raw = raw_params(6000)
    m, ref = make_model(raw), make_ref(raw)
    cam = orbit_camera(1, 320, 240, 300.0)
    ups = Hn.upstream_grads(cam.height, cam.width, seed=3)
    st = Hn.settings_for(cam, 3, DEV)

    def render(xyz, feats, op, sc, rot, seg):
        means2D = torch.zeros_like(xyz, requires_grad=True)
        color, radii, depth, alpha, segment = GaussianRasterizer(st)(
            means3D=xyz, means2D=means2D, shs=feats, colors_precomp=None, segments=seg, opacities=op, scales=sc,
            rotations=rot, cov3D_precomp=None)
        torch.autograd.backward([color, depth, alpha, segment],
                                [ups["color"].to(DEV), ups["depth"].to(DEV), ups["alpha"].to(DEV),
                                 ups["segment"].to(DEV)])
        return color

    before = dict(GM.BACKWARD_PATHS)
    c1 = render(m.get_xyz, m.get_features, m.get_opacity, m.get_scaling, m.get_rotation, m.get_segment)
    assert GM.BACKWARD_PATHS["zero_copy"] == before["zero_copy"] + 1, GM.BACKWARD_PATHS
    # the same render on detached leaves gives dL/d(activated), fed to the oracle's autograd
    with torch.no_grad():
        leaves = [t.detach().clone().requires_grad_(True) for t in
                  (m.get_xyz, m.get_features, m.get_opacity, m.get_scaling, m.get_rotation, m.get_segment)]
    c2 = render(*leaves)
    assert torch.equal(c1, c2)
    keys = ["xyz", "features", "opacity", "scaling", "rotation", "segment"]
    ref.backward_from_activated({k: t.grad.cpu() for k, t in zip(keys, leaves)})
    for name in GROUPS:
        close(m._spec.group(m._arena.grad, name), ref.params[name].grad, 5e-6,
              rot_atol(leaves[4].grad, raw["rotation"]) if name == "rotation" else 1e-9, f"d{name}")


@pytest.mark.parametrize("sh_degree", [3, 0])
def test_adam_matches_torch_adam(gpu_available, sh_degree):
    raw = raw_params(3001, sh_degree=sh_degree)
    m, ref = make_model(raw, sh_degree), make_ref(raw)
    m.spatial_lr_scale = 1.0
    m.training_setup(_Args)
    lrs = {g["name"]: g["lr"] for g in m.optimizer.param_groups}
    ref.training_setup(lrs)
    g = torch.Generator().manual_seed(11)
    keys = ["xyz", "features", "opacity", "scaling", "rotation", "segment"]
    for it in range(1, 7):
        lr = m.update_learning_rate(it * 1000)
        ref.set_lr("xyz", lr)
        grads = {k: torch.randn(v.shape, generator=g) * 1e-2 for k, v in ref.activated().items()}
        grads["opacity"][::5] = 0.0  # zero-gradient rows: m, v decay only
        outs = [m.get_xyz, m.get_features, m.get_opacity, m.get_scaling, m.get_rotation, m.get_segment]
        torch.autograd.backward(outs, [grads[k].to(DEV) for k in keys])
        m.optimizer.step()
        m.optimizer.zero_grad(set_to_none=True)
        ref.backward_from_activated(grads)
        ref.step()
    for name in GROUPS:
        close(m.group_view(name), ref.params[name], 1e-5, 1e-6, name)
        st = ref.optimizer.state[ref.params[name]]
        close(m._spec.group(m.optimizer.exp_avg, name), st["exp_avg"], 1e-5, 1e-9, f"{name}.exp_avg")
        close(m._spec.group(m.optimizer.exp_avg_sq, name), st["exp_avg_sq"], 1e-5, 1e-14, f"{name}.exp_avg_sq")
    # the activated buffer the step wrote equals a fresh activation of the new parameters
    with torch.no_grad():
        a = ref.activated()
        close(m.get_opacity, a["opacity"], 1e-5, 1e-7, "opacity after step")
        close(m.get_scaling, a["scaling"], 1e-5, 1e-9, "scaling after step")
        close(m.get_rotation, a["rotation"], 1e-5, 1e-7, "rotation after step")
    # torch.optim.Adam state_dict interoperability (checkpoints of capture()/restore())
    sd = ref.optimizer.state_dict()
    m2 = make_model({k: ref.params[k].detach() for k in GROUPS}, sh_degree)
    m2.spatial_lr_scale = 1.0
    m2.training_setup(_Args)
    m2.optimizer.load_state_dict(sd)
    for name in GROUPS:
        close(m2._spec.group(m2.optimizer.exp_avg_sq, name), ref.optimizer.state[ref.params[name]]["exp_avg_sq"],
              0, 0, f"{name} loaded exp_avg_sq")
    back = torch.optim.Adam([{"params": [torch.nn.Parameter(ref.params[n].detach().clone())], "name": n, "lr": 0.0}
                             for n in GROUPS], lr=0.0, eps=1e-15)
    back.load_state_dict(m2.optimizer.state_dict())
    assert float(back.state_dict()["state"][0]["step"]) == 6.0


def test_densify_stats(gpu_available):
    from gsr_train import GaussianModel  # noqa: F401
    raw = raw_params(2500)
    m, ref = make_model(raw), make_ref(raw)
    m.training_setup(_Args)
    g = torch.Generator().manual_seed(5)
    for _ in range(3):
        radii = torch.randint(-1, 40, (2500,), generator=g, dtype=torch.int32)
        radii[radii < 0] = 0
        dm2 = torch.randn(2500, 3, generator=g) * 1e-3
        m.update_densification_stats(dm2.to(DEV), radii.to(DEV))
        ref.densify_stats(dm2, radii)
    close(m.max_radii2D, ref.max_radii2D, 0, 0, "max_radii2D")
    close(m.denom, ref.denom, 0, 0, "denom")
    close(m.xyz_gradient_accum, ref.xyz_gradient_accum, 1e-6, 1e-12, "xyz_gradient_accum")
    # the reference signature: add_densification_stats(viewspace_point_tensor, update_filter)
    vis = torch.rand(2500, generator=g) > 0.5
    vp = torch.zeros(2500, 3, device=DEV, requires_grad=True)
    vp.grad = (torch.randn(2500, 3, generator=g) * 1e-3).to(DEV)
    before = m.denom.clone()
    m.add_densification_stats(vp, vis.to(DEV))
    assert torch.equal((m.denom - before).squeeze(1).cpu() > 0, vis)


def _trained_pair(P, seed=0):
    """GPU model + CPU oracle after two identical Adam steps (non-zero moments)."""
    raw = raw_params(P, seed=seed)
    g = torch.Generator().manual_seed(seed + 1)
    raw["scaling"] = raw["scaling"] + torch.randn(P, 3, generator=g) * 0.8  # spread around the clone/split edge
    op = torch.rand(P, 1, generator=g)
    op[::7] = 0.002  # below min_opacity
    raw["opacity"] = torch.logit(op)
    m, ref = make_model(raw), make_ref(raw)
    m.spatial_lr_scale = 1.0
    m.training_setup(_Args)
    ref.training_setup({gr["name"]: gr["lr"] for gr in m.optimizer.param_groups})
    keys = ["xyz", "features", "opacity", "scaling", "rotation", "segment"]
    for _ in range(2):
        grads = {k: torch.randn(v.shape, generator=g) * 1e-2 for k, v in ref.activated().items()}
        torch.autograd.backward([m.get_xyz, m.get_features, m.get_opacity, m.get_scaling, m.get_rotation,
                                 m.get_segment], [grads[k].to(DEV) for k in keys])
        m.optimizer.step()
        m.optimizer.zero_grad()
        ref.backward_from_activated(grads)
        ref.step()
    return m, ref, g


def _compare_state(m, ref, what):
    """Parameters, Adam moments and statistics in the reference's row order.  The
    two Adam steps before already differ by fp32 rounding (GPU vs CPU), so rows are
    compared at the Adam tolerance; statistics exactly."""
    for name in GROUPS:
        a, b = m.group_view(name), ref.params[name].detach()
        assert a.shape == b.shape, f"{what} {name}: {tuple(a.shape)} vs {tuple(b.shape)}"
        # Adam steps already differ by rounding (see test_adam_matches_torch_adam): 1e-5
        close(a, b, 1e-5, 1e-6, f"{what} {name}")
        st = ref.optimizer.state[ref.params[name]]
        close(m._spec.group(m.optimizer.exp_avg, name), st["exp_avg"], 1e-5, 1e-9, f"{what} {name}.exp_avg")
        close(m._spec.group(m.optimizer.exp_avg_sq, name), st["exp_avg_sq"], 1e-5, 1e-14,
              f"{what} {name}.exp_avg_sq")
    close(m.xyz_gradient_accum, ref.xyz_gradient_accum, 0, 0, f"{what} accum")
    close(m.denom, ref.denom, 0, 0, f"{what} denom")
    close(m.max_radii2D, ref.max_radii2D, 0, 0, f"{what} max_radii2D")


def test_densify_and_prune_matches_reference(gpu_available):
    from oracle.train_oracle import RefDensify
    P = 20000
    m, ref, g = _trained_pair(P)
    # statistics: mean gradient ~ half above threshold, some never-visible (0/0 -> 0)
    accum = (torch.rand(P, 1, generator=g) * 4e-4)
    denom = torch.randint(0, 4, (P, 1), generator=g).float()
    accum[denom == 0] = 0.0
    m.xyz_gradient_accum.copy_(accum.to(DEV))
    m.denom.copy_(denom.to(DEV))
    ref.xyz_gradient_accum, ref.denom = accum.clone(), denom.clone()
    extent, max_grad, min_op = 1.2, 2e-4 / 2, 0.005
    gen = torch.Generator(device=DEV).manual_seed(1234)
    counts = m.densify_and_prune(max_grad, min_op, extent, 20, generator=gen)
    assert counts[1] > 100 and counts[3] > 100, counts  # both clones and splits happen
    gen2 = torch.Generator(device=DEV).manual_seed(1234)
    normals = torch.empty((2 * counts[3], 3), device=DEV).normal_(0.0, 1.0, generator=gen2).cpu()
    RefDensify.densify_and_prune(ref, max_grad, min_op, extent, 20, _Args.percent_dense, normals)
    assert m.num_points == ref.params["xyz"].shape[0] == counts[0] + counts[1] + 2 * counts[2]
    _compare_state(m, ref, "densify_and_prune")
    # the model keeps training after the rebuild (layout, optimizer views, activations)
    with torch.no_grad():
        close(m.get_scaling, torch.exp(ref.params["scaling"].detach()), 2e-6, 1e-12, "scaling after densify")
    grads = {k: torch.randn(v.shape, generator=g) * 1e-2 for k, v in ref.activated().items()}
    keys = ["xyz", "features", "opacity", "scaling", "rotation", "segment"]
    torch.autograd.backward([m.get_xyz, m.get_features, m.get_opacity, m.get_scaling, m.get_rotation,
                             m.get_segment], [grads[k].to(DEV) for k in keys])
    m.optimizer.step()
    ref.backward_from_activated(grads)
    ref.step()
    for name in GROUPS:
        close(m.group_view(name), ref.params[name].detach(), 2e-5, 2e-6, f"step after densify {name}")


def test_prune_points_and_reset_opacity(gpu_available):
    from oracle.train_oracle import RefDensify
    P = 5000
    m, ref, g = _trained_pair(P, seed=4)
    mask = torch.rand(P, generator=g) < 0.3
    stats = torch.rand(P, 1, generator=g)
    m.xyz_gradient_accum.copy_(stats.to(DEV))
    ref.xyz_gradient_accum = stats.clone()
    m.prune_points(mask.to(DEV))
    RefDensify.prune(ref, mask)
    _compare_state(m, ref, "prune_points")
    m.reset_opacity()
    with torch.no_grad():
        op = torch.sigmoid(ref.params["opacity"])
        new = torch.log(torch.min(op, torch.ones_like(op) * 0.01) / (1 - torch.min(op, torch.ones_like(op) * 0.01)))
    close(m._opacity, new, 1e-5, 1e-6, "reset_opacity")
    assert float(m._spec.group(m.optimizer.exp_avg, "opacity").abs().max()) == 0.0
    assert float(m._spec.group(m.optimizer.exp_avg, "xyz").abs().max()) > 0.0
