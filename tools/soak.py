"""Soak run of the drop-in API (GPU): N forward+backward steps of the metric scene through
rasterize_gaussians (the default route: the C++ autograd function), checking that device memory,
the caching allocator's reservation and the host's resident set stay flat and that the outputs stay
bit-identical step after step.  usage: python tools/soak.py [steps] [config]"""
import os
import resource
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "3d_gaussian_magic_change-segment_3dgs_amd")]
import torch  # noqa: E402

import diff_gaussian_rasterization as dgr  # noqa: E402
from diff_gaussian_rasterization import _C  # noqa: E402
from gsr_tools.scene import config_scene_and_camera  # noqa: E402


def rss_mb():
    with open("/proc/self/statm") as f:
        return int(f.read().split()[1]) * resource.getpagesize() / 2**20


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    cfg = sys.argv[2] if len(sys.argv) > 2 else "mt"
    dev = torch.device("cuda", 0)
    scene, cam = config_scene_and_camera(cfg)
    leaf = lambda t: t.to(dev).contiguous().requires_grad_(True)
    means3D, shs, opac = leaf(scene.means3D), leaf(scene.shs), leaf(scene.opacities)
    scales, rots, segs = leaf(scene.scales), leaf(scene.rotations), leaf(scene.segments)
    means2D = torch.zeros_like(means3D, requires_grad=True)
    E = torch.empty(0, device=dev)
    st = dgr.GaussianRasterizationSettings(
        image_height=cam.height, image_width=cam.width, tanfovx=cam.tanfovx, tanfovy=cam.tanfovy,
        bg=torch.zeros(3, device=dev), scale_modifier=1.0, viewmatrix=cam.world_view_transform.to(dev),
        projmatrix=cam.full_proj_transform.to(dev), sh_degree=scene.sh_degree, campos=cam.camera_center.to(dev),
        prefiltered=False, debug=False)
    gen = torch.Generator().manual_seed(1)
    ups = [(torch.randn(c, cam.height, cam.width, generator=gen) * 1e-3).to(dev) for c in (3, 1, 1, 2)]
    params = [means3D, shs, opac, scales, rots, segs, means2D]

    def step():
        color, radii, depth, alpha, segment = dgr.rasterize_gaussians(means3D, means2D, shs, E, segs, opac, scales,
                                                                      rots, E, st)
        g = torch.autograd.grad([color, depth, alpha, segment], params, ups)
        return color, g

    ref_c, ref_g = step()
    ref_c, ref_g = ref_c.detach().clone(), [x.clone() for x in ref_g]
    route = "C++ autograd" if _C._HOST_AUTOGRAD is not None else "Python autograd"
    marks, t0 = [], time.perf_counter()
    for i in range(1, steps + 1):
        c, g = step()
        if i % (steps // 10) == 0:
            torch.cuda.synchronize()
            same = torch.equal(c, ref_c) and all(torch.equal(a, b) for a, b in zip(g, ref_g))
            marks.append((i, torch.cuda.memory_allocated() / 2**20, torch.cuda.memory_reserved() / 2**20, rss_mb(),
                          same))
            print(f"step {i:6d}: allocated {marks[-1][1]:8.1f} MiB  reserved {marks[-1][2]:8.1f} MiB  "
                  f"host RSS {marks[-1][3]:8.1f} MiB  bit-identical to step 0: {same}", flush=True)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    first, last = marks[0], marks[-1]
    print(f"{cfg}: {steps} steps in {el:.2f} s ({steps / el:.1f} views/s) through the {route} route; "
          f"allocated {first[1]:.1f} -> {last[1]:.1f} MiB, reserved {first[2]:.1f} -> {last[2]:.1f} MiB, "
          f"host RSS {first[3]:.1f} -> {last[3]:.1f} MiB; every checkpoint bit-identical: {all(m[4] for m in marks)}")
    assert all(m[4] for m in marks), "outputs drifted"
    assert last[1] <= first[1] + 1.0 and last[2] <= first[2] + 1.0, "device memory grew"
    assert last[3] <= first[3] + 64.0, "host memory grew"


if __name__ == "__main__":
    main()
