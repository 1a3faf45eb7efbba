"""Parity budget study: the HIP path (whatever libgsr GSR_LIBRARY points at) against the
CPU oracle evaluated with (a) the kernels' own blend exp and (b) the C library's expf
(an exp independent of gsr, the closest stand-in for the reference's CUDA expf).

For every case prints one JSON line with, per output:
  images : max |d| / max(1, |ref|) and the fraction of pixels above 1e-5
  grads  : max |d| / max|ref| (scale-free, per tensor) and the fraction of elements above
           1e-5 * max|ref|
  n_contrib mismatching pixels, num_rendered difference.
Usage: python tools/parity_budget.py [case ...]   (cases: c1 sh3 bgmod large c2 mt c3 c5)
"""
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "3d_gaussian_magic_change-segment_3dgs_amd"), os.path.join(ROOT, "tests")]
import numpy as np
import torch

import harness as Hn
from oracle import oracle as O
from gsr_tools.scene import config_scene_and_camera, synthetic_scene, orbit_camera


def img_stats(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    e = np.abs(a - b) / np.maximum(1.0, np.abs(b))
    return {"max": float(e.max()), "frac": float((e > 1e-5).reshape(e.shape[0], -1).any(0).mean())}


def grad_stats(a, b):
    a, b = np.asarray(a, np.float64).reshape(b.shape), np.asarray(b, np.float64)
    s = float(np.abs(b).max()) if b.size else 0.0
    if s == 0.0:
        return {"max": float(np.abs(a).max()) if a.size else 0.0, "frac": 0.0, "ref_max": 0.0}
    e = np.abs(a - b) / s
    return {"max": float(e.max()), "frac": float((e > 1e-5).mean()), "ref_max": s}


def compare(g, r):
    out = {"n_contrib_mismatch": int((g["n_contrib"].astype(np.uint32) != r["n_contrib"]).sum()),
           "num_rendered_diff": int(g["num_rendered"]) - int(r["num_rendered"])}
    for k in ("color", "depth", "alpha", "segment"):
        out[k] = img_stats(g[k], r[k])
    for k, ref in r["grads"].items():
        if k not in g["grads"]:
            continue
        a = np.asarray(g["grads"][k]).reshape(ref.shape)
        b = ref
        if k == "dmeans2D":
            a, b = a[:, :2], b[:, :2]
        out[k] = grad_stats(a, b)
    return out


def cases():
    c = {}
    c["c1"] = lambda: (*config_scene_and_camera("c1"), {})
    c["sh3"] = lambda: (synthetic_scene(20000, sh_degree=3, seed=3), orbit_camera(1, 333, 250, 300.0), {})
    c["bgmod"] = lambda: (synthetic_scene(20000, sh_degree=3, seed=3), orbit_camera(1, 333, 250, 300.0),
                          dict(bg=(0.2, 0.5, 0.9), scale_modifier=0.7))
    c["large"] = lambda: (synthetic_scene(400, sh_degree=2, seed=9, log_scale=math.log(0.4), log_scale_std=0.3),
                          orbit_camera(3, 300, 200, 250.0), {})
    for name in ("c2", "mt", "c3", "c5"):
        c[name] = (lambda n: lambda: (*config_scene_and_camera(n), {}))(name)
    return c


def main():
    torch.cuda.init()
    from diff_gaussian_rasterization import _C
    lib = os.environ.get("GSR_LIBRARY", "default")
    names = sys.argv[1:] or ["c1", "sh3", "bgmod", "large", "c2", "mt"]
    C = cases()
    for name in names:
        scene, cam, kw = C[name]()
        grads = Hn.upstream_grads(cam.height, cam.width)
        t0 = time.time()
        g = Hn.run_gsr(scene, cam, grads=grads, **kw)
        t1 = time.time()
        res = {"case": name, "lib": os.path.basename(lib), "P": scene.P, "W": cam.width, "H": cam.height,
               "I": int(g["num_rendered"])}
        modes = os.environ.get("PB_MODES", "same_exp,libm").split(",")
        r64 = None
        for mode in modes:
            if mode == "acc32":  # the reference's own fp32 accumulation-order noise vs the exact sums
                O.set_acc32(True)
                r32 = Hn.run_oracle(O, scene, cam, grads=grads, **kw)
                O.set_acc32(False)
                if r64 is None:
                    r64 = Hn.run_oracle(O, scene, cam, grads=grads, **kw)
                res[mode] = compare(r32, r64)
                del r32
                continue
            O.set_exp_libm(mode == "libm")
            r = Hn.run_oracle(O, scene, cam, grads=grads, **kw)
            res[mode] = compare(g, r)
            if mode == "same_exp":
                r64 = r
            del r
        O.set_exp_libm(False)
        r64 = None
        res["t_gsr_s"], res["t_total_s"] = round(t1 - t0, 2), round(time.time() - t0, 2)
        print(json.dumps(res), flush=True)
        del g


if __name__ == "__main__":
    main()
