"""Host-side time of one fwd+bwd step through the drop-in GaussianRasterizer (GPU).

Stamps perf_counter_ns around the C entry points (gsr_forward, gsr_backward: the ctypes route),
around the C++ binding's calls (GSR_HOST_AUTOGRAD=0), or reads the stamps the C++ autograd function
takes itself (the default route), and prints, per phase, the median host microseconds over the timed steps:
  py_fwd_pre   step start -> gsr_forward entry (Python wrapper, argument checks, allocations)
  c_fwd        inside gsr_forward (launches + the num_rendered wait)
  fwd_to_bwd   gsr_forward exit -> gsr_backward entry (autograd, backward wrapper)
  c_bwd        inside gsr_backward (launches)
  py_bwd_post  gsr_backward exit -> step end
The GPU idles before the backward render when py_fwd_pre + c_fwd + fwd_to_bwd exceeds the
GPU time of the forward.  usage: python tools/host_overhead.py [config] [steps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "3d_gaussian_magic_change-segment_3dgs_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import diff_gaussian_rasterization as dgr  # noqa: E402
from diff_gaussian_rasterization import _C  # noqa: E402
from gsr_tools.scene import config_scene_and_camera  # noqa: E402


class _Stamped:
    def __init__(self, fn, log, tag):
        self.fn, self.log, self.tag = fn, log, tag
        self.argtypes, self.restype = fn.argtypes, fn.restype

    def __call__(self, *a):
        self.log.append((self.tag + "_in", time.perf_counter_ns()))
        r = self.fn(*a)
        self.log.append((self.tag + "_out", time.perf_counter_ns()))
        return r


class _Host:
    """The C++ host binding (gsr_host) with its two entry points stamped; its lib_ns() counter
    gives the part of each call spent inside libgsr (launches + the num_rendered wait)."""

    def __init__(self, host, log):
        self._h, self._log = host, log

    def _call(self, tag, fn, *a):
        self._log.append((tag + "_in", time.perf_counter_ns()))
        l0 = self._h.lib_ns()
        r = fn(*a)
        lib = self._h.lib_ns() - l0
        t = time.perf_counter_ns()
        self._log.append((tag + "_lib", lib))
        self._log.append((tag + "_out", t))
        return r

    def rasterize_gaussians(self, *a):
        return self._call("f", self._h.rasterize_gaussians, *a)

    def rasterize_gaussians_backward(self, *a):
        return self._call("b", self._h.rasterize_gaussians_backward, *a)

    def __getattr__(self, k):
        return getattr(self._h, k)


class _Lib:
    def __init__(self, lib, log):
        self._lib, self._log = lib, log
        self.gsr_forward = _Stamped(lib.gsr_forward, log, "f")
        self.gsr_backward = _Stamped(lib.gsr_backward, log, "b")

    def __getattr__(self, k):
        return getattr(self._lib, k)


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "mt"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    dev = torch.device("cuda", 0)
    scene, cam = config_scene_and_camera(cfg)
    leaf = lambda t: t.to(dev).contiguous().requires_grad_(True)
    means3D, shs, opac = leaf(scene.means3D), leaf(scene.shs), leaf(scene.opacities)
    scales, rots, segs = leaf(scene.scales), leaf(scene.rotations), leaf(scene.segments)
    means2D = torch.zeros_like(means3D, requires_grad=True)
    E = torch.empty(0, device=dev)
    H, W = cam.height, cam.width
    st = dgr.GaussianRasterizationSettings(
        image_height=H, image_width=W, tanfovx=cam.tanfovx, tanfovy=cam.tanfovy, bg=torch.zeros(3, device=dev),
        scale_modifier=1.0, viewmatrix=cam.world_view_transform.to(dev), projmatrix=cam.full_proj_transform.to(dev),
        sh_degree=scene.sh_degree, campos=cam.camera_center.to(dev), prefiltered=False, debug=False)
    gen = torch.Generator().manual_seed(1)
    ups = [(torch.randn(c, H, W, generator=gen) * 1e-3).to(dev) for c in (3, 1, 1, 2)]
    params = [means3D, shs, opac, scales, rots, segs, means2D]
    log = []
    # routes: the C++ autograd function (stamps taken inside it), the Python autograd function over
    # the C++ binding (GSR_HOST_AUTOGRAD=0) or over ctypes (GSR_HOST_EXT=0)
    route = "autograd" if _C._HOST_AUTOGRAD is not None else "cpp" if _C._HOST is not None else "ctypes"
    cpp = route != "ctypes"
    if route == "cpp":
        _C._HOST = _Host(_C._HOST, log)
    elif route == "ctypes":
        _C._lib = _Lib(_C._lib, log)

    def step():
        log.append(("s", time.perf_counter_ns()))
        color, radii, depth, alpha, segment = dgr.rasterize_gaussians(means3D, means2D, shs, E, segs, opac, scales,
                                                                      rots, E, st)
        g = torch.autograd.grad([color, depth, alpha, segment], params, ups)
        log.append(("e", time.perf_counter_ns()))
        return g

    for _ in range(10):
        step()
    torch.cuda.synchronize()
    log.clear()
    if os.environ.get("HOST_CPROFILE"):  # function-level host profile of the same loop
        import cProfile
        import pstats
        pr = cProfile.Profile()
        pr.enable()
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        pr.disable()
        pstats.Stats(pr).sort_stats("tottime").print_stats(35)
        log.clear()
    if route == "autograd":
        _C._HOST_AUTOGRAD.stamps(True)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / steps * 1e6
    if route == "autograd":
        # the C++ stamps (kind, t_in, lib_ns, t_out) in call order, merged into the step log
        stamps = _C._HOST_AUTOGRAD.stamps(False)
        fw, bw = [x for x in stamps if x[0] == 0], [x for x in stamps if x[0] == 1]
        ss, es = [v for k, v in log if k == "s"], [v for k, v in log if k == "e"]
        log = []
        for s_, f, b, e in zip(ss, fw, bw, es):
            log += [("s", s_), ("f_in", f[1]), ("f_lib", f[2]), ("f_out", f[3]), ("b_in", b[1]), ("b_lib", b[2]),
                    ("b_out", b[3]), ("e", e)]
    ph = {k: [] for k in ("py_fwd_pre", "c_fwd", "fwd_to_bwd", "c_bwd", "py_bwd_post", "total",
                          "host_excl_lib")}
    i = 0
    if cpp:
        # C++ route: the stamps bracket the binding's calls; lib = the time inside libgsr.  The
        # binding's own host work is counted in py_fwd_pre / fwd_to_bwd / py_bwd_post, so that the
        # phases mean what they mean for the ctypes route (host time outside the libgsr calls).
        names = ["s", "f_in", "f_lib", "f_out", "b_in", "b_lib", "b_out", "e"]
        while i < len(log):
            seq = log[i:i + 8]
            i += 8
            if [t for t, _ in seq] != names:
                continue
            t = dict(seq)
            fh = (t["f_out"] - t["f_in"] - t["f_lib"]) / 1e3  # binding's host work around gsr_forward
            bh = (t["b_out"] - t["b_in"] - t["b_lib"]) / 1e3
            ph["py_fwd_pre"].append((t["f_in"] - t["s"]) / 1e3 + fh)
            ph["c_fwd"].append(t["f_lib"] / 1e3)
            ph["fwd_to_bwd"].append((t["b_in"] - t["f_out"]) / 1e3 + bh)
            ph["c_bwd"].append(t["b_lib"] / 1e3)
            ph["py_bwd_post"].append((t["e"] - t["b_out"]) / 1e3)
            ph["total"].append((t["e"] - t["s"]) / 1e3)
    else:
        while i < len(log):
            seq = log[i:i + 6]
            i += 6
            if [t for t, _ in seq] != ["s", "f_in", "f_out", "b_in", "b_out", "e"]:
                continue
            t = [v for _, v in seq]
            for k, a, b in (("py_fwd_pre", 0, 1), ("c_fwd", 1, 2), ("fwd_to_bwd", 2, 3), ("c_bwd", 3, 4),
                            ("py_bwd_post", 4, 5), ("total", 0, 5)):
                ph[k].append((t[b] - t[a]) / 1e3)
    ph["host_excl_lib"] = [a + b + c for a, b, c in zip(ph["py_fwd_pre"], ph["fwd_to_bwd"], ph["py_bwd_post"])]
    names = {"autograd": "C++ autograd function (gsr_host)", "cpp": "C++ (gsr_host) under the Python autograd "
             "function", "ctypes": "ctypes"}
    print(f"{cfg}: {len(ph['total'])} steps, wall {wall:.1f} us/step (GPU-synchronised loop); host binding: "
          f"{names[route]}")
    for k, v in ph.items():
        print(f"  {k:12s} median {np.median(v):8.1f} us  p90 {np.percentile(v, 90):8.1f}")


if __name__ == "__main__":
    main()
