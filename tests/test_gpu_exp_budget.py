"""Parity against an INDEPENDENT exp: the HIP path (blending with gsr_expf) vs the CPU
oracle blending with the C library's expf (glibc, correctly rounded in practice) --
the closest stand-in here for the reference's CUDA expf (forward.cu:351,
backward.cu:547; specified at 2 ulp, not reproducible bit for bit off NVIDIA parts).

Two different correctly-rounded-or-nearly exps disagree in the last bit on a small
fraction of inputs.  The blend thresholds (alpha >= 1/255, T(1-alpha) >= 1e-4) turn a
last-bit alpha difference into a different decision for a pixel now and then, and the
backward's T = 1 - sum(alpha T) recovery (backward.cu:468) amplifies it by 1/T_final;
so some gradient elements move by more than 1e-5 of the tensor maximum ("knife-edge
outliers") whichever exp either side uses.  The budget below bounds their fraction
and size per output; it is the DESIGN.md s4 budget, with about 2x headroom over the
values measured on MI355X (profiles/round2_exp_budget_gsr_expf.jsonl).  The same study
run with the hardware exp (-DGSR_FAST_EXP: v_exp_f32(x log2e), faithful but not
correctly rounded; profiles/round2_exp_budget_fast_exp.jsonl) breaks this budget at
C2 and the metric config (outlier fraction 2x, max 3.5x, image error 300x), which is
why the kernels keep gsr_expf.
"""
import math

import numpy as np
import pytest

import harness as Hn
from gsr_tools.scene import config_scene_and_camera, synthetic_scene, orbit_camera

pytestmark = pytest.mark.gpu

# case -> (grad outlier fraction, grad max normwise error, image max error, n_contrib mismatch fraction)
BUDGET = {
    "c1": (1e-3, 1e-4, 2e-5, 1e-4),
    "sh3": (1e-3, 1e-4, 2e-5, 1e-4),
    "large": (0.15, 1e-3, 2e-5, 1e-4),   # 400 screen-filling Gaussians: every pixel sees ~100 of them
    "c2": (0.05, 5e-4, 2e-5, 1e-4),
    "mt": (0.02, 5e-4, 2e-5, 1e-4),
}


def _case(name):
    if name == "sh3":
        return synthetic_scene(20000, sh_degree=3, seed=3), orbit_camera(1, 333, 250, 300.0)
    if name == "large":
        return (synthetic_scene(400, sh_degree=2, seed=9, log_scale=math.log(0.4), log_scale_std=0.3),
                orbit_camera(3, 300, 200, 250.0))
    return config_scene_and_camera(name)


@pytest.mark.parametrize("name", list(BUDGET))
def test_knife_edge_budget_vs_libm_exp(gpu_available, oracle_mod, name):
    frac_b, max_b, img_b, nc_b = BUDGET[name]
    scene, cam = _case(name)
    grads = Hn.upstream_grads(cam.height, cam.width)
    g = Hn.run_gsr(scene, cam, grads=grads)
    oracle_mod.set_exp_libm(True)
    try:
        r = Hn.run_oracle(oracle_mod, scene, cam, grads=grads)
    finally:
        oracle_mod.set_exp_libm(False)
    # binning does not involve exp: still bit-exact
    assert g["num_rendered"] == r["num_rendered"]
    np.testing.assert_array_equal(g["point_list"].astype(np.uint32), r["point_list"])
    nc = float((g["n_contrib"].astype(np.uint32) != r["n_contrib"]).mean())
    assert nc <= nc_b, f"n_contrib: {nc:.2e} of pixels differ (budget {nc_b:.0e})"
    for k in ("color", "depth", "alpha", "segment"):
        a, b = g[k].astype(np.float64), r[k].astype(np.float64)
        e = float((np.abs(a - b) / np.maximum(1.0, np.abs(b))).max())
        assert e <= img_b, f"{k}: max error {e:.2e} (budget {img_b:.0e})"
    report = {}
    for k, ref in r["grads"].items():
        if k not in g["grads"]:
            continue
        a = np.asarray(g["grads"][k], np.float64).reshape(ref.shape)
        b = ref.astype(np.float64)
        if k == "dmeans2D":
            a, b = a[:, :2], b[:, :2]
        e = np.abs(a - b) / float(np.abs(b).max())
        frac, mx = float((e > 1e-5).mean()), float(e.max())
        report[k] = (frac, mx)
        assert frac <= frac_b, f"{k}: {frac:.2e} of elements above 1e-5 * max|ref| (budget {frac_b:.0e})"
        assert mx <= max_b, f"{k}: max normwise error {mx:.2e} (budget {max_b:.0e})"
    print(name, {k: f"frac {f:.1e} max {m:.1e}" for k, (f, m) in report.items()})
