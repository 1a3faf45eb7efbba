"""CPU oracle of the training step around the rasterizer.

TEST INFRASTRUCTURE ONLY: imported by tests/ (and bench.py's cpu_baseline leg),
never by the product package.

It restates the reference's Gaussian container (scene/gaussian_model.py) the
reference's way -- seven separate fp32 nn.Parameters on the CPU, activations as
torch ops (:34-43,100-127), and the very optimizer the reference builds,
torch.optim.Adam(groups, lr=0.0, eps=1e-15) (:162-172) -- so it is pinned by
construction to the reference's arithmetic (the Adam step *is* torch's).
Densification statistics follow train.py:168-172 / gaussian_model.py:523-526.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

GROUPS = ("xyz", "f_dc", "f_rest", "opacity", "segment", "scaling", "rotation")


class RefGaussians:
    """scene/gaussian_model.py's parameter set, CPU fp32."""

    def __init__(self, xyz, f_dc, f_rest, opacity, segment, scaling, rotation):
        t = lambda x: nn.Parameter(torch.as_tensor(x, dtype=torch.float32).detach().cpu().clone())
        self.params = {"xyz": t(xyz), "f_dc": t(f_dc), "f_rest": t(f_rest), "opacity": t(opacity),
                       "segment": t(segment), "scaling": t(scaling), "rotation": t(rotation)}
        P = self.params["xyz"].shape[0]
        self.xyz_gradient_accum = torch.zeros((P, 1))
        self.denom = torch.zeros((P, 1))
        self.max_radii2D = torch.zeros(P)
        self.optimizer = None

    # gaussian_model.py:100-127
    def activated(self):
        p = self.params
        return {"xyz": p["xyz"], "features": torch.cat((p["f_dc"], p["f_rest"]), dim=1),
                "opacity": torch.sigmoid(p["opacity"]), "scaling": torch.exp(p["scaling"]),
                "rotation": F.normalize(p["rotation"]), "segment": torch.sigmoid(p["segment"])}

    # gaussian_model.py:158-172
    def training_setup(self, lrs):
        """lrs: {group name: lr} (the values training_setup derives from OptimizationParams)."""
        groups = [{"params": [self.params[n]], "lr": lrs[n], "name": n} for n in GROUPS]
        self.optimizer = torch.optim.Adam(groups, lr=0.0, eps=1e-15)

    def set_lr(self, name, lr):
        for g in self.optimizer.param_groups:
            if g["name"] == name:
                g["lr"] = lr

    def backward_from_activated(self, grads):
        """Backpropagate gradients given w.r.t. the activated tensors (what the
        rasterizer returns) into the raw parameters (.grad), through torch autograd."""
        act = self.activated()
        outs, gs = [], []
        for k, g in grads.items():
            if g is not None:
                outs.append(act[k])
                gs.append(torch.as_tensor(g, dtype=torch.float32).cpu().reshape(act[k].shape))
        torch.autograd.backward(outs, gs)

    def step(self):
        self.optimizer.step()
        self.optimizer.zero_grad(set_to_none=True)

    # train.py:170-172 + gaussian_model.py:523-526
    @torch.no_grad()
    def densify_stats(self, dmeans2D, radii):
        vis = radii > 0
        self.max_radii2D[vis] = torch.max(self.max_radii2D[vis], radii[vis].float())
        self.xyz_gradient_accum[vis] += torch.norm(dmeans2D[vis, :2], dim=-1, keepdim=True)
        self.denom[vis] += 1


# ---- densification (gaussian_model.py:362-521), CPU restatement ---------------------
# The optimizer bookkeeping follows the reference: pruning indexes the Adam moments
# of each param group with the keep-mask (_prune_optimizer :378-396), growing
# appends zero moments (cat_tensors_to_optimizer :359-384); "step" is untouched.

def _build_rotation(r):
    """utils/general_utils.py:86-107."""
    norm = torch.sqrt(r[:, 0] * r[:, 0] + r[:, 1] * r[:, 1] + r[:, 2] * r[:, 2] + r[:, 3] * r[:, 3])
    q = r / norm[:, None]
    w, x, y, z = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    R = torch.zeros((q.shape[0], 3, 3))
    R[:, 0, 0] = 1 - 2 * (y * y + z * z)
    R[:, 0, 1] = 2 * (x * y - w * z)
    R[:, 0, 2] = 2 * (x * z + w * y)
    R[:, 1, 0] = 2 * (x * y + w * z)
    R[:, 1, 1] = 1 - 2 * (x * x + z * z)
    R[:, 1, 2] = 2 * (y * z - w * x)
    R[:, 2, 0] = 2 * (x * z - w * y)
    R[:, 2, 1] = 2 * (y * z + w * x)
    R[:, 2, 2] = 1 - 2 * (x * x + y * y)
    return R


def _swap_param(opt, name, new_tensor, moment_fn):
    """Replace group `name`'s parameter, transforming its Adam moments with moment_fn."""
    for group in opt.param_groups:
        if group["name"] != name:
            continue
        old = group["params"][0]
        st = opt.state.get(old, None)
        newp = nn.Parameter(new_tensor.requires_grad_(True))
        if st is not None:
            st["exp_avg"] = moment_fn(st["exp_avg"])
            st["exp_avg_sq"] = moment_fn(st["exp_avg_sq"])
            del opt.state[old]
            opt.state[newp] = st
        group["params"][0] = newp
        return newp


class RefDensify:
    """Mixin-style functions over a RefGaussians (with training_setup done)."""

    @staticmethod
    def prune(g, mask):
        keep = ~mask
        for n in GROUPS:
            g.params[n] = _swap_param(g.optimizer, n, g.params[n].detach()[keep], lambda t: t[keep])
        g.xyz_gradient_accum = g.xyz_gradient_accum[keep]
        g.denom = g.denom[keep]
        g.max_radii2D = g.max_radii2D[keep]

    @staticmethod
    def postfix(g, new):
        for n in GROUPS:
            ext = new[n]
            g.params[n] = _swap_param(g.optimizer, n, torch.cat((g.params[n].detach(), ext), dim=0),
                                      lambda t, ext=ext: torch.cat((t, torch.zeros_like(ext)), dim=0))
        P = g.params["xyz"].shape[0]
        g.xyz_gradient_accum = torch.zeros((P, 1))
        g.denom = torch.zeros((P, 1))
        g.max_radii2D = torch.zeros(P)

    @staticmethod
    def clone(g, grads, thr, extent, percent_dense):
        scaling = torch.exp(g.params["scaling"].detach())
        sel = (torch.norm(grads, dim=-1) >= thr) & (torch.max(scaling, dim=1).values <= percent_dense * extent)
        RefDensify.postfix(g, {n: g.params[n].detach()[sel] for n in GROUPS})

    @staticmethod
    def split(g, grads, thr, extent, percent_dense, normals, N=2):
        P = g.params["xyz"].shape[0]
        padded = torch.zeros(P)
        padded[:grads.shape[0]] = grads.squeeze()
        scaling = torch.exp(g.params["scaling"].detach())
        sel = (padded >= thr) & (torch.max(scaling, dim=1).values > percent_dense * extent)
        ns = int(sel.sum())
        stds = scaling[sel].repeat(N, 1)
        samples = normals[:N * ns].reshape(N * ns, 3) * stds  # torch.normal(0, std) = z * std (+ 0)
        rots = _build_rotation(g.params["rotation"].detach()[sel]).repeat(N, 1, 1)
        new = {"xyz": torch.bmm(rots, samples.unsqueeze(-1)).squeeze(-1) + g.params["xyz"].detach()[sel].repeat(N, 1),
               "scaling": torch.log(scaling[sel].repeat(N, 1) / (0.8 * N))}
        for n in ("f_dc", "f_rest", "opacity", "segment", "rotation"):
            t = g.params[n].detach()[sel]
            new[n] = t.repeat(N, *([1] * (t.dim() - 1)))
        RefDensify.postfix(g, new)
        RefDensify.prune(g, torch.cat((sel, torch.zeros(N * ns, dtype=torch.bool))))
        return ns

    @staticmethod
    def densify_and_prune(g, max_grad, min_opacity, extent, max_screen_size, percent_dense, normals):
        grads = g.xyz_gradient_accum / g.denom
        grads[grads.isnan()] = 0.0
        RefDensify.clone(g, grads, max_grad, extent, percent_dense)
        RefDensify.split(g, grads, max_grad, extent, percent_dense, normals)
        prune = (torch.sigmoid(g.params["opacity"].detach()) < min_opacity).squeeze()
        if max_screen_size:
            big_vs = g.max_radii2D > max_screen_size
            big_ws = torch.exp(g.params["scaling"].detach()).max(dim=1).values > 0.1 * extent
            prune = torch.logical_or(torch.logical_or(prune, big_vs), big_ws)
        RefDensify.prune(g, prune)


# ---- PLY (gaussian_model.py:207-224 save_ply, :270-315 load_ply) ---------------------
# The reference writes with plyfile (absent here: parity unpinned against plyfile
# itself; the byte layout below restates the PLY spec as plyfile emits it for an
# all-'f4' vertex element: ascii header, `format binary_little_endian 1.0`,
# `property float <name>` per attribute, then the packed little-endian rows).

def ply_attribute_matrix(xyz, f_dc, f_rest, opacity, segment, scaling, rotation):
    """The [P, F] float32 matrix save_ply concatenates (normals are zeros; f_dc /
    f_rest are transposed to channel-major before flattening)."""
    import numpy as np
    a = lambda t: torch.as_tensor(t).detach().float().cpu()
    P = a(xyz).shape[0]
    fdc = a(f_dc).transpose(1, 2).flatten(start_dim=1)
    frest = a(f_rest).transpose(1, 2).flatten(start_dim=1)
    cols = [a(xyz), torch.zeros(P, 3), fdc, frest, a(opacity).reshape(P, 1), a(segment), a(scaling), a(rotation)]
    return np.concatenate([c.numpy() for c in cols], axis=1).astype(np.float32)


def ply_reference_bytes(names, matrix, fmt="binary_little_endian", prop_type="float"):
    """Bytes of a PLY file with one vertex element (plyfile's layout)."""
    import numpy as np
    head = ["ply", f"format {fmt} 1.0", f"element vertex {matrix.shape[0]}"]
    head += [f"property {prop_type} {n}" for n in names] + ["end_header"]
    out = ("\n".join(head) + "\n").encode("ascii")
    if fmt == "ascii":
        return out + "".join(" ".join(repr(float(v)) for v in row) + "\n" for row in matrix).encode("ascii")
    np_t = {"float": "f4", "double": "f8"}[prop_type]
    end = "<" if fmt == "binary_little_endian" else ">"
    return out + np.ascontiguousarray(matrix, dtype=end + np_t).tobytes()
