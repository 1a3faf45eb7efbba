import os, sys, math
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "3d_gaussian_magic_change-segment_3dgs_amd"), os.path.join(ROOT, "tests")]
import numpy as np, torch
import harness as Hn
from oracle import oracle as O
from gsr_tools.scene import Scene, make_camera, focal2fov
cam = make_camera(np.eye(3), np.array([0.0, 0.0, 2.0]), 17, 9, focal2fov(20.0, 17), focal2fov(20.0, 9))
grads = Hn.upstream_grads(cam.height, cam.width)
worst = []
for seed in range(300):
    gen = torch.Generator().manual_seed(seed)
    scene = Scene(torch.tensor([[0.01, -0.02, 0.0]]), torch.rand(1, 16, 3, generator=gen) * 0.1, torch.tensor([[0.8]]),
                  torch.tensor([[0.05, 0.08, 0.03]]), torch.tensor([[0.9, 0.1, 0.3, -0.2]]) / math.sqrt(0.95),
                  torch.tensor([[0.3, 0.7]]), 3)
    g = Hn.run_gsr(scene, cam, grads=grads, want_state=False)
    O.set_acc32(False); r = Hn.run_oracle(O, scene, cam, grads=grads)
    O.set_acc32(True); r32 = Hn.run_oracle(O, scene, cam, grads=grads); O.set_acc32(False)
    e = {}
    for k in r["grads"]:
        if k not in g["grads"]: continue
        a = np.asarray(g["grads"][k], np.float64).reshape(r["grads"][k].shape); b = r["grads"][k].astype(np.float64); c = r32["grads"][k].astype(np.float64)
        if k == "dmeans2D": a, b, c = a[:, :2], b[:, :2], c[:, :2]
        sc = np.abs(b).max()
        if sc == 0: continue
        e[k] = (np.abs(a - b).max() / sc, np.abs(c - b).max() / sc)
    k = max(e, key=lambda k: e[k][0])
    worst.append((e[k][0], seed, k, e[k][1]))
worst.sort(reverse=True)
print("worst gsr err (err, seed, tensor, fp32-order err):", [(f"{w[0]:.2e}", w[1], w[2], f"{w[3]:.2e}") for w in worst[:6]])
print("count > 1e-5:", sum(w[0] > 1e-5 for w in worst), " fp32-order > 1e-5:", sum(w[3] > 1e-5 for w in worst))
