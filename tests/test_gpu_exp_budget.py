"""Parity against an INDEPENDENT exp, stated precisely (VERDICT r4 Next #5, r5 Next #1).

The HIP path blends with gsr_expf, which the CPU oracle shares bit for bit, so every other
parity test compares identical exps.  The reference's CUDA expf (forward.cu:351,
backward.cu:547) is specified at 2 ulp and cannot run here.  Three stand-ins for it, each a
mode of the oracle ("L" below):
  * libm: the C library's expf (glibc: < 1 ulp, almost always correctly rounded);
  * jit1 / jit2: gsr_expf moved by -1..+1 / -2..+2 ulp per (Gaussian, pixel) by a fixed hash
    (oracle set_exp_jitter), the same in forward and backward -- an exp of CUDA's specified
    accuracy, and a wider perturbation than glibc's.
Two exps that differ in the last bits reach the outputs through exactly two mechanisms, which
this test separates and bounds:

1. Flipped blend decisions.  alpha >= 1/255 and T(1 - alpha) >= 1e-4 (forward.cu:352-359)
   are thresholds: a last-bit alpha can change which list positions a pixel blends or where it
   stops.  The oracle hashes every pixel's decision sequence (oracle_get "dhash": the blended
   positions and the terminating one); pixels whose hash differs between the two exps are
   the flipped pixels.  They are counted and reported (0-5 per view at these configs);
   everything below is asserted on the other pixels (a flipped pixel's upstream gradients
   are zeroed, which removes its every gradient term).
2. The backward's T_final recovery.  backward.cu:468 starts each pixel's back-to-front replay
   from T_final = 1 - (weight sum) and divides by (1 - alpha) per contributor.  A weight sum
   that differs in its last bits (|d alpha_out| <= 1e-6 here) becomes a relative error of
   ~1e-7 / T_final in every T the replay reconstructs; dense scenes have T_final < 1e-3 on
   most pixels, so 0.1-15 % of gradient elements of the reference itself move by more than
   1e-5 of the tensor maximum when only the exp changes (measured below, "unpinned").
   Running L's backward from the HIP forward's weight sums (oracle set_weight_sums)
   removes exactly this mechanism.

Asserted per case (c1, sh3, a screen-filling 'large' case, and the BASELINE configs C2, the
metric scene, C3 and C5 at full size) and per exp mode, with G = the oracle with gsr_expf,
L = the oracle in that mode run from G's weight sums (mechanism 2 pinned), both on the
unflipped pixels:
  * point_list / num_rendered bit-exact (binning involves no exp);
  * n_contrib identical on every unflipped pixel; flipped pixels <= 1e-4 of the image;
  * images within 1e-5 * max(1, |ref|) on unflipped pixels, and the weight sums within 1e-6;
  * gradients, scale-free (|d| <= tol * max|ref| per element of each tensor, as
    test_gpu_parity.py), ZERO elements above:
      (i)   HIP vs G: 1e-5 -- the fp32 summation-order noise test_gpu_parity.py bounds
            (dscales / drot: 4e-5, below);
      (ii)  G vs L: 1e-5 -- the exp's direct effect once mechanisms 1 and 2 are removed --
            except dscales / drot: 4e-5.  Those two leave the per-Gaussian chain
            dconic -> dcov2D -> dcov3D -> (scale, rotation) (backward.cu:141-341), whose
            cancellations amplify a last-bit change of the summed conic gradient: measured
            (profiles/round6_exp_modes.txt) every other tensor stays below 1e-6 in every mode,
            dscales / drot reach 0.8e-5 (libm) to 2.7e-5 (+-2 ulp) at C3 / C5;
      (iii) HIP vs L: (i) + (ii), so nothing is left unexplained;
  * the unpinned deviation (L from its own weight sums) is reported per tensor, with a
    regression guard of about 1.5x the worst value measured over the seven cases in that mode
    (profiles/round6_exp_modes.txt, worst at the 'large' case: libm 3.4e-4 -> guard 5.5e-4;
    jitter 1.5e-3 -> 2.3e-3; round 5's single guard was 1e-3).
"""
import math

import numpy as np
import pytest
import torch

import harness as Hn
from contract_cases import case_scene

pytestmark = pytest.mark.gpu

CASES = ["c1", "sh3", "large", "c2", "mt", "c3", "c5"]
MODES = ["libm", "jit1", "jit2"]
KEYS = ("dmeans2D", "dopacity", "dmeans3D", "dsh", "dscales", "drot", "dsegments")
JITTER_SEED = 12345
# dscales / drot: 4e-5 -- the cancellations of the dconic -> dcov3D -> (scale, rotation) chain
# (backward.cu:141-341) move them most: the reference's own fp32 atomic-order deviation reaches
# 1.7e-5 of the tensor maximum there at C3 (tests/test_gpu_parity.py assert_grad_parity)
TOL_I = {k: (4e-5 if k in ("dscales", "drot") else 1e-5) for k in KEYS}
TOL_II = {k: (4e-5 if k in ("dscales", "drot") else 1e-5) for k in KEYS}
# unpinned guard per mode: ~1.5x the worst measured (profiles/round6_exp_modes.txt)
UNPINNED_GUARD = {"libm": 5.5e-4, "jit1": 2.3e-3, "jit2": 2.3e-3}


def _set_mode(O, mode):
    O.set_exp_libm(mode == "libm")
    jit = mode.startswith("jit")
    O.set_exp_jitter(JITTER_SEED if jit else 0, ulps=int(mode[3:]) if jit else 1)


def _normwise(a, b, k):
    a, b = np.asarray(a, np.float64).reshape(b.shape), b.astype(np.float64)
    if k == "dmeans2D":
        a, b = a[:, :2], b[:, :2]
    return np.abs(a - b) / max(float(np.abs(b).max()), 1e-30)


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("name", CASES)
def test_independent_exp_precise(gpu_available, oracle_mod, name, mode):
    O = oracle_mod
    scene, cam = case_scene(name)
    H, W = cam.height, cam.width
    grads = Hn.upstream_grads(H, W)
    # decisions under both exps (forward only for gsr_expf: the HIP path's decisions are the
    # oracle's bit for bit, tests/test_gpu_parity.py)
    _set_mode(O, "none")
    own = O.run_scene(scene, cam)
    _set_mode(O, mode)
    try:
        lib = O.run_scene(scene, cam)
        flipped = (own.get("dhash") != lib.get("dhash")).reshape(H, W)
        keep = ~flipped
        km = torch.from_numpy(keep)[None]
        masked = {k: (v * km).contiguous() for k, v in grads.items()}
        g = Hn.run_gsr(scene, cam, grads=masked)
        assert g["num_rendered"] == lib.num_rendered
        np.testing.assert_array_equal(g["point_list"].astype(np.uint32), lib.get("point_list"))
        nc_lib = lib.get("n_contrib").reshape(H, W)
        assert np.array_equal(g["n_contrib"].astype(np.uint32)[keep], nc_lib[keep]), "n_contrib on an unflipped pixel"
        assert flipped.mean() <= 1e-4, f"{int(flipped.sum())} flipped pixels"
        img = 0.0
        for k, ref in (("color", lib.color), ("depth", lib.depth), ("alpha", lib.alpha), ("segment", lib.segment)):
            e = np.abs(g[k].astype(np.float64) - ref) / np.maximum(1.0, np.abs(ref))
            img = max(img, float(e[:, keep].max()) if keep.any() else 0.0)
        assert img <= 1e-5, f"image error {img:.2e} on unflipped pixels"
        dw = float(np.abs(g["alpha"][0].astype(np.float64) - lib.alpha[0])[keep].max()) if keep.any() else 0.0
        assert dw <= 1e-6, f"weight sums differ by {dw:.2e}"
        ups = [masked[k].numpy() for k in ("color", "segment", "depth", "alpha")]
        free = lib.backward(*ups)                # libm backward from its own weight sums
        lib.set_weight_sums(own.alpha)           # ... and from gsr_expf's (mechanism 2 pinned)
        pinned = lib.backward(*ups)
    finally:
        _set_mode(O, "none")
    G = own.backward(*ups)
    del own
    checks = {"(i) HIP vs G": (g["grads"], G, TOL_I), "(ii) G vs L": (G, pinned, TOL_II),
              "(iii) HIP vs L": (g["grads"], pinned, {k: TOL_I[k] + v for k, v in TOL_II.items()})}
    rep, rep_free = {c: {} for c in checks}, {}
    for k in KEYS:
        if k not in g["grads"]:
            continue
        for c, (x, y, tol) in checks.items():
            t = tol[k] if isinstance(tol, dict) else tol
            e = _normwise(x[k], y[k], k)
            rep[c][k] = (int((e > t).sum()), float(e.max()), t)
        f = _normwise(g["grads"][k], free[k], k)
        rep_free[k] = (float((f > 1e-5).mean()), float(f.max()))
    print(f"\n{name} [{mode}]: flipped pixels {int(flipped.sum())} of {flipped.size}; image (unflipped) {img:.1e}; "
          f"|d weight sum| {dw:.1e}")
    for c, r in rep.items():
        print(f"  {c:15s}: " + ", ".join(f"{k} {n} > {t:.0e} (max {m:.1e})" for k, (n, m, t) in r.items()))
    print(f"  unpinned HIP vs {mode}: " + ", ".join(f"{k} {fr:.2%} > 1e-5 (max {m:.1e})" for k, (fr, m) in rep_free.items()))
    for c, r in rep.items():
        for k, (n, m, t) in r.items():
            assert n == 0, f"{c}: {k}: {n} elements above {t:.0e} * max|ref| (max {m:.2e})"
    for k, (fr, m) in rep_free.items():
        assert m <= UNPINNED_GUARD[mode], f"{k}: unpinned max normwise deviation {m:.2e}"
