"""GaussianAdam: the reference's torch.optim.Adam over the seven Gaussian param
groups (scene/gaussian_model.py:162-172), as one fused HIP pass over the arena.

Same surface the reference's training code touches: `param_groups` (list of
dicts with "name", "lr", "betas", "eps", "params"), `step()`, `zero_grad(
set_to_none=True)`, `state_dict()` / `load_state_dict()` in torch.optim.Adam's
format (so a checkpoint's optimizer state from `GaussianModel.capture()`,
gaussian_model.py:64-79, loads either way).  The moments are two arenas shaped
like the parameter arena; step() is one gsr_adam_step launch that also refreshes
the activated buffer the next render consumes.
"""
import torch

from . import _C


class GaussianAdam:
    def __init__(self, model, groups, lr=0.0, eps=1e-15, betas=(0.9, 0.999), weight_decay=0.0, amsgrad=False):
        if weight_decay != 0.0 or amsgrad:
            raise ValueError("GaussianAdam implements the reference's plain Adam (no weight decay / amsgrad)")
        self.model = model
        self.defaults = dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=0.0, amsgrad=False)
        self.param_groups = []
        seen = set()
        for g in groups:
            name = g.get("name")
            if name not in _C.GROUP_NAMES or name in seen:
                raise ValueError(f"GaussianAdam: group name must be one of {_C.GROUP_NAMES} (once), got {name!r}")
            seen.add(name)
            d = dict(self.defaults)
            d.update({k: v for k, v in g.items() if k != "params"})
            d["params"] = [model.group_view(name)]
            self.param_groups.append(d)
        self.steps = {g["name"]: 0 for g in self.param_groups}
        arena = model._arena.data
        self.exp_avg = torch.zeros_like(arena)
        self.exp_avg_sq = torch.zeros_like(arena)

    # ---- torch.optim.Optimizer surface -------------------------------------------------
    def _hyper(self):
        h = _C.AdamHyper()
        betas = {tuple(g["betas"]) for g in self.param_groups}
        epss = {float(g["eps"]) for g in self.param_groups}
        if len(betas) > 1 or len(epss) > 1:
            raise ValueError("GaussianAdam: all groups must share betas and eps (one fused launch)")
        b1, b2 = next(iter(betas)) if betas else self.defaults["betas"]
        h.beta1, h.beta2 = float(b1), float(b2)
        h.one_minus_beta1, h.one_minus_beta2 = 1 - b1, 1 - b2  # python doubles, as torch passes them
        h.eps = next(iter(epss)) if epss else self.defaults["eps"]
        by_name = {g["name"]: g for g in self.param_groups}
        for k, name in enumerate(_C.GROUP_NAMES):
            g = by_name.get(name)
            if g is None:
                h.skip[k] = 1
                continue
            self.steps[name] += 1
            t = self.steps[name]
            # torch _multi_tensor_adam (capturable=False): python-float bias corrections
            bc1 = 1 - b1 ** t
            bc2 = 1 - b2 ** t
            h.step_size[k] = float(g["lr"]) / bc1
            h.bc2_sqrt[k] = bc2 ** 0.5
        return h

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        m = self.model
        grad = m._arena.grad
        if grad is None:  # torch skips parameters without a gradient
            return loss
        if grad.shape != m._arena.shape or not grad.is_contiguous() or grad.dtype != torch.float32:
            raise RuntimeError("GaussianAdam: arena gradient has the wrong shape/layout")
        _C.adam_step(m._spec, m._arena.data, grad, self.exp_avg, self.exp_avg_sq, m._act, self._hyper())
        m._params_changed(act_fresh=True)
        return loss

    def zero_grad(self, set_to_none=True):
        g = self.model._arena.grad
        if g is None:
            return
        if set_to_none:
            self.model._arena.grad = None
        else:
            g.zero_()

    @property
    def state(self):
        """{param view: {"step", "exp_avg", "exp_avg_sq"}} like torch.optim.Adam.state
        (views into the moment arenas)."""
        spec = self.model._spec
        out = {}
        for g in self.param_groups:
            n = g["name"]
            out[g["params"][0]] = {"step": torch.tensor(float(self.steps[n])),
                                   "exp_avg": spec.group(self.exp_avg, n), "exp_avg_sq": spec.group(self.exp_avg_sq, n)}
        return out

    def state_dict(self):
        spec = self.model._spec
        state, groups = {}, []
        for i, g in enumerate(self.param_groups):
            n = g["name"]
            if self.steps[n] > 0:
                state[i] = {"step": torch.tensor(float(self.steps[n])),
                            "exp_avg": spec.group(self.exp_avg, n).clone(),
                            "exp_avg_sq": spec.group(self.exp_avg_sq, n).clone()}
            d = {k: v for k, v in g.items() if k != "params"}
            d["params"] = [i]
            groups.append(d)
        return {"state": state, "param_groups": groups}

    @torch.no_grad()
    def load_state_dict(self, sd):
        """Accepts this class's state_dict or a torch.optim.Adam one built over the
        reference's seven nn.Parameters (matched by group name)."""
        spec = self.model._spec
        groups = sd["param_groups"]
        by_name = {g["name"]: g for g in self.param_groups}
        for sg in groups:
            name = sg.get("name")
            if name not in by_name:
                raise ValueError(f"load_state_dict: unknown group {name!r}")
            g = by_name[name]
            for k, v in sg.items():
                if k != "params":
                    g[k] = tuple(v) if k == "betas" else v
            idx = sg["params"][0]
            st = sd["state"].get(idx)
            if st is None:
                self.steps[name] = 0
                spec.group(self.exp_avg, name).zero_()
                spec.group(self.exp_avg_sq, name).zero_()
                continue
            self.steps[name] = int(round(float(st["step"])))
            for key, dst in (("exp_avg", self.exp_avg), ("exp_avg_sq", self.exp_avg_sq)):
                view = spec.group(dst, name)
                src = st[key]
                if tuple(src.shape) != tuple(view.shape):
                    raise ValueError(f"load_state_dict: {name}.{key} has shape {tuple(src.shape)}, "
                                     f"expected {tuple(view.shape)}")
                view.copy_(src.to(view.device, torch.float32))

    # ---- arena maintenance used by GaussianModel (densification / resets) ------------
    def _resize(self, exp_avg, exp_avg_sq):
        self.exp_avg, self.exp_avg_sq = exp_avg, exp_avg_sq
        for g in self.param_groups:
            g["params"] = [self.model.group_view(g["name"])]

    def _reset_group(self, name):
        """replace_tensor_to_optimizer (gaussian_model.py:362-376): moments of one
        group to zero, step kept."""
        spec = self.model._spec
        spec.group(self.exp_avg, name).zero_()
        spec.group(self.exp_avg_sq, name).zero_()


def bias_corrections(beta1, beta2, step):
    """(1 - beta1^t, sqrt(1 - beta2^t)) as torch.optim.Adam computes them (float64)."""
    return 1 - beta1 ** step, (1 - beta2 ** step) ** 0.5
