"""Where does a gradient element exceed the scale-free 1e-5 bound?  Runs one config view
through gsr and the oracle (exact fp64 sums, fp32 atomic-order emulation), and for each
gradient tensor prints the worst elements: gsr / oracle / fp32-order values, the
Gaussian's radius, tiles touched and screen position.

usage: python tools/grad_outlier_diag.py CONFIG VIEW N_VIEWS SEED"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "3d_gaussian_magic_change-segment_3dgs_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import harness as Hn  # noqa: E402
from oracle import oracle as O  # noqa: E402
from gsr_tools.scene import config_scene_and_camera  # noqa: E402


def main():
    cfg, view, nv, seed = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
    O.build()
    scene, cam = config_scene_and_camera(cfg, view_index=view, n_views=nv)
    grads = Hn.upstream_grads(cam.height, cam.width, seed=seed)
    g = Hn.run_gsr(scene, cam, grads=grads)
    O.set_acc32(False)
    r = Hn.run_oracle(O, scene, cam, grads=grads)
    O.set_acc32(True)
    r32 = Hn.run_oracle(O, scene, cam, grads=grads)
    O.set_acc32(False)
    for k, ref in r["grads"].items():
        if k not in g["grads"]:
            continue
        a = np.asarray(g["grads"][k], np.float64).reshape(ref.shape)
        b = ref.astype(np.float64)
        c = np.asarray(r32["grads"][k], np.float64).reshape(ref.shape)
        if k == "dmeans2D":
            a, b, c = a[:, :2], b[:, :2], c[:, :2]
        sc = np.abs(b).max()
        e = np.abs(a - b) / sc
        e32 = np.abs(c - b) / sc
        print(f"{k:10s} max|ref| {sc:.3e}  gsr max {e.max():.2e} n>1e-5 {(e > 1e-5).sum()}  "
              f"fp32-order max {e32.max():.2e} n>1e-5 {(e32 > 1e-5).sum()}")
        flat = np.argsort(e.reshape(-1))[::-1][:3]
        for f in flat:
            i = np.unravel_index(f, e.shape)
            gi = i[0]
            print(f"   elem {i}: gsr {a[i]:+.6e} oracle {b[i]:+.6e} fp32-order {c[i]:+.6e} err {e[i]:.2e} "
                  f"(fp32-order err {e32[i]:.2e}) radius {g['radii'][gi]} tiles {g['tiles_touched'][gi]} "
                  f"xy {g['rec'].reshape(-1, 16)[gi, :2]} opacity {float(scene.opacities[gi]):.3f} "
                  f"scales {scene.scales[gi].numpy()}")


if __name__ == "__main__":
    main()
