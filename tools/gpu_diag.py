"""One-shot GPU diagnostic: HIP path vs CPU oracle on several cases, printing
every comparison (does not stop at the first mismatch)."""
import math
import os
import sys
import time
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "3d_gaussian_magic_change-segment_3dgs_amd"), os.path.join(ROOT, "tests")]
import numpy as np
import torch

from gsr_tools.scene import config_scene_and_camera, synthetic_scene, orbit_camera
from oracle import oracle as O
import harness as Hn


def cmp_case(name, scene, cam, **kw):
    print(f"=== {name}: P={scene.P} {cam.width}x{cam.height} deg={scene.sh_degree}", flush=True)
    grads = Hn.upstream_grads(cam.height, cam.width)
    t0 = time.time()
    g = Hn.run_gsr(scene, cam, grads=grads, **kw)
    t1 = time.time()
    r = Hn.run_oracle(O, scene, cam, grads=grads, **kw)
    t2 = time.time()
    print(f"  gsr {t1-t0:.2f}s oracle {t2-t1:.2f}s  I gsr={g['num_rendered']} oracle={r['num_rendered']}")
    print("  radii equal:", np.array_equal(g["radii"], r["radii"]), " n_diff", int((g["radii"] != r["radii"]).sum()))
    print("  tiles_touched equal:", np.array_equal(g["tiles_touched"].astype(np.uint32), r["tiles_touched"]))
    if g["num_rendered"] == r["num_rendered"]:
        print("  point_list equal:", np.array_equal(g["point_list"].astype(np.uint32), r["point_list"]),
              " ranges equal:", np.array_equal(g["ranges"].astype(np.uint32), r["ranges"]))
    nc = (g["n_contrib"].astype(np.uint32) != r["n_contrib"]).sum()
    print("  n_contrib mismatches:", int(nc), "of", r["n_contrib"].size)
    rec = g["rec"].reshape(-1, 16)
    vis = r["radii"] > 0
    if vis.any():
        print("  means2D exact:", np.array_equal(rec[vis, 0:2], r["means2D"].reshape(-1, 2)[vis]),
              " conic/opac exact:", np.array_equal(rec[vis][:, [2, 3, 4, 5]], r["conic_opacity"].reshape(-1, 4)[vis]),
              " depth exact:", np.array_equal(rec[vis, 6], r["depths"][vis]))
        if kw.get("colors_precomp") is None:
            print("  rgb exact:", np.array_equal(rec[vis][:, [8, 9, 10]], r["rgb"].reshape(-1, 3)[vis]),
                  " clamped exact:", np.array_equal(g["clamped"][vis],
                                                    (r["clamped"].reshape(-1, 3) * [1, 2, 4]).sum(1)[vis]))
    for k in ("color", "depth", "alpha", "segment"):
        d = np.abs(g[k] - r[k])
        print(f"  {k}: max|d|={d.max():.3e} rel={Hn.tol_report(g[k], r[k]):.3e} max|ref|={np.abs(r[k]).max():.3e}")
    for k, v in r["grads"].items():
        if k not in g["grads"]:
            continue
        a = g["grads"][k].reshape(v.shape) if g["grads"][k] is not None else None
        if a is None:
            print(f"  grad {k}: None on gsr side")
            continue
        if k == "dsh":
            a = a.reshape(v.shape)
        d = np.abs(a - v)
        print(f"  grad {k}: max|d|={d.max():.3e} tol={Hn.tol_report(a, v):.3e} max|ref|={np.abs(v).max():.3e}")


def main():
    torch.cuda.init()
    print(torch.cuda.get_device_name(0), flush=True)
    from diff_gaussian_rasterization import _C
    print("lib", _C.version())
    cases = []
    sc, cam = config_scene_and_camera("c1")
    cases.append(("c1", sc, cam, {}))
    sc = synthetic_scene(20000, sh_degree=3, seed=3)
    cam = orbit_camera(1, 333, 250, 300.0)
    cases.append(("sh3_ragged", sc, cam, {}))
    cases.append(("sh3_bg_mod", sc, cam, dict(bg=(0.2, 0.5, 0.9), scale_modifier=0.7)))
    sc1 = synthetic_scene(20000, sh_degree=3, seed=4)
    cases.append(("sh3_as_deg1", sc1, cam, dict(sh_degree=1)))
    cols = torch.rand(20000, 3, generator=torch.Generator().manual_seed(5))
    cases.append(("colors_precomp", sc, cam, dict(colors_precomp=cols)))
    # cov3D precomp from the scene's scale/rot (torch restatement)
    cases.append(("no_segments", sc, cam, dict(use_segments=False)))
    if os.environ.get("DIAG_MT_PARITY"):
        sc_mt, cam_mt = config_scene_and_camera("mt")
        cases.append(("mt", sc_mt, cam_mt, {}))
    only = os.environ.get("DIAG_CASES")
    for name, s, c, kw in cases:
        if only and name not in only.split(","):
            continue
        try:
            cmp_case(name, s, c, **kw)
        except Exception:
            traceback.print_exc()
    if os.environ.get("DIAG_NO_MT"):
        return
    # full-size timing
    sc, cam = config_scene_and_camera("mt")
    from diff_gaussian_rasterization import _RasterizeGaussians
    st = Hn.settings_for(cam, 3, "cuda")
    dev = "cuda"
    leaf = lambda t: t.to(dev).requires_grad_(True)
    m3, sh, op, scl, rot, seg = (leaf(sc.means3D), leaf(sc.shs), leaf(sc.opacities), leaf(sc.scales),
                                 leaf(sc.rotations), leaf(sc.segments))
    m2 = torch.zeros_like(m3, requires_grad=True)
    gr = {k: v.to(dev) for k, v in Hn.upstream_grads(cam.height, cam.width).items()}
    E = torch.Tensor([])
    for it in range(8):
        torch.cuda.synchronize(); t0 = time.time()
        color, radii, depth, alpha, segment = _RasterizeGaussians.apply(m3, m2, sh, E, seg, op, scl, rot, E, st)
        torch.cuda.synchronize(); t1 = time.time()
        torch.autograd.backward([color, depth, alpha, segment], [gr["color"], gr["depth"], gr["alpha"], gr["segment"]])
        torch.cuda.synchronize(); t2 = time.time()
        print(f"mt iter {it}: fwd {1e3*(t1-t0):.2f} ms bwd {1e3*(t2-t1):.2f} ms I={color.grad_fn.num_rendered if color.grad_fn else -1}", flush=True)
        for t in (m3, m2, sh, op, scl, rot, seg):
            t.grad = None


if __name__ == "__main__":
    main()
