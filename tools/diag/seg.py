import sys, os
sys.path[:0] = ["/root/repo", "/root/repo/3d_gaussian_magic_change-segment_3dgs_amd", "/root/repo/tests"]
import numpy as np
import harness as Hn
from gsr_tools.scene import synthetic_scene, orbit_camera
from diff_gaussian_rasterization import _C
scene, cam = synthetic_scene(60000, sh_degree=3, seed=41), orbit_camera(2, 640, 360, 400.0)
grads = Hn.upstream_grads(cam.height, cam.width)
res = {}
for rows in (1, 0):
    for ck in (256, 0):
        for rep in (0, 1):
            _C.set_option("rows_binning", rows); _C.set_option("bwd_ckpt", ck)
            res[(rows, ck, rep)] = Hn.run_gsr(scene, cam, grads=grads)
T = 40 * 23
for key, g in res.items():
    d = g["n_contrib_tiles"].reshape(-1, 256).max(1)
    print(key, "depth max", d.max(), "tiles >= 320:", int((d >= 320).sum()), "sched", g["tile_order"][T:T+4])
base = res[(1, 0, 0)]["grads"]
for key, g in res.items():
    print(key, {k: float(np.abs(g["grads"][k] - base[k]).max()) for k in base})
