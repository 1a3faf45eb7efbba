"""Compare GPU gradient error with the reference's own fp32-accumulation noise
(oracle in fp32-accumulate mode vs exact-sum mode) on the hard scenes."""
import math, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "3d_gaussian_magic_change-segment_3dgs_amd"), os.path.join(ROOT, "tests")]
import numpy as np, torch
import harness as Hn
from oracle import oracle as O
from gsr_tools.scene import synthetic_scene, orbit_camera, config_scene_and_camera

def stats(a, b):
    a = np.asarray(a, np.float64); b = np.asarray(b, np.float64)
    sc = max(1.0, np.abs(b).max())
    e = np.abs(a - b) / sc
    return e.max(), (e > 1e-5).mean()

def run(name, scene, cam, **kw):
    grads = Hn.upstream_grads(cam.height, cam.width)
    g = Hn.run_gsr(scene, cam, grads=grads, want_state=False, **kw)
    O.set_acc32(False); r64 = Hn.run_oracle(O, scene, cam, grads=grads, **kw)
    O.set_acc32(True); r32 = Hn.run_oracle(O, scene, cam, grads=grads, **kw)
    O.set_acc32(False)
    O.set_exp_libm(True); rl = Hn.run_oracle(O, scene, cam, grads=grads, **kw)
    O.set_exp_libm(False)
    print(f"== {name}")
    for k, ref in r64["grads"].items():
        if k not in g["grads"]: continue
        a = g["grads"][k].reshape(ref.shape); b32 = r32["grads"][k]; bl = rl["grads"][k]
        if k == "dmeans2D": a, ref2, b32, bl = a[:, :2], ref[:, :2], b32[:, :2], bl[:, :2]
        else: ref2 = ref
        eg, fg = stats(a, ref2); eo, fo = stats(b32, ref2); el, fl = stats(bl, ref2)
        print(f"  {k:10s} gpu: max {eg:.2e} frac>1e-5 {fg:.2e} | fp32-order noise: {eo:.2e} | libm-exp noise: max {el:.2e} frac {fl:.2e}")

torch.cuda.init()
g = torch.Generator().manual_seed(6)
sc = synthetic_scene(20000, sh_degree=3, seed=3); cam = orbit_camera(1, 333, 250, 300.0)
A = torch.randn(sc.P, 3, 3, generator=g) * 0.02
S = A @ A.transpose(1, 2) + torch.eye(3) * 1e-5
cov = torch.stack([S[:, 0, 0], S[:, 0, 1], S[:, 0, 2], S[:, 1, 1], S[:, 1, 2], S[:, 2, 2]], 1).contiguous()
run("cov3d", sc, cam, cov3D_precomp=cov)
run("large", synthetic_scene(400, sh_degree=2, seed=9, log_scale=math.log(0.4), log_scale_std=0.3), orbit_camera(3, 300, 200, 250.0))
sc, cam = config_scene_and_camera("c1"); run("c1", sc, cam)
sc, cam = config_scene_and_camera("mt"); run("mt", sc, cam)
