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
