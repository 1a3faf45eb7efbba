import sys
import os; R=os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))); sys.path[:0]=[R, R+'/tests', R+'/3d_gaussian_magic_change-segment_3dgs_amd']
import numpy as np, torch
import harness as Hn
from oracle import oracle as O
from contract_cases import case_scene
import test_gpu_exp_budget as T
name, mode = sys.argv[1], sys.argv[2]
scene, cam = case_scene(name)
H, W = cam.height, cam.width
grads = Hn.upstream_grads(H, W)
T._set_mode(O, "none")
own = O.run_scene(scene, cam)
T._set_mode(O, mode)
lib = O.run_scene(scene, cam)
flipped = (own.get("dhash") != lib.get("dhash")).reshape(H, W)
keep = ~flipped
km = torch.from_numpy(keep)[None]
masked = {k: (v * km).contiguous() for k, v in grads.items()}
ups = [masked[k].numpy() for k in ("color", "segment", "depth", "alpha")]
free = lib.backward(*ups)
lib.set_weight_sums(own.alpha)
pinned = lib.backward(*ups)
T._set_mode(O, "none")
G = own.backward(*ups)
for k in T.KEYS:
    e = T._normwise(G[k], pinned[k], k)
    print(k, int((e > 1e-5).sum()), e.max())
import hashlib
h = lambda a: hashlib.md5(np.ascontiguousarray(a).tobytes()).hexdigest()[:12]
print("scene", h(scene.means3D.numpy()), h(scene.scales.numpy()), h(scene.rotations.numpy()), h(scene.opacities.numpy()), h(scene.shs.numpy()))
print("own", h(own.color), h(own.alpha), "lib", h(lib.alpha))
print("G", {k: h(v) for k, v in G.items()})
print("pinned", {k: h(v) for k, v in pinned.items()})
