"""Wave-level loop statistics of the render kernels (instrumented build).

Build:  make -C 3d_gaussian_magic_change-segment_3dgs_amd/csrc OUT=$PWD/build/diag/libgsr_stats.so \
            HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -fvisibility=hidden -DGSR_STATS"
Run:    python tools/render_stats.py [config]      (GPU; loads the instrumented library)
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("GSR_LIBRARY", os.path.join(ROOT, "build", "diag", "libgsr_stats.so"))
sys.path[:0] = [ROOT, os.path.join(ROOT, "3d_gaussian_magic_change-segment_3dgs_amd"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402

from diff_gaussian_rasterization import _C  # noqa: E402
from gsr_tools.scene import config_scene_and_camera  # noqa: E402
import harness as Hn  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "mt"
    lib = _C._lib
    lib.gsr_stats_read.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    buf = (ctypes.c_ulonglong * 32)()
    scene, cam = config_scene_and_camera(cfg)
    grads = Hn.upstream_grads(cam.height, cam.width)
    Hn.run_gsr(scene, cam, grads=grads, want_state=False)  # warm-up
    torch.cuda.synchronize()
    lib.gsr_stats_read(buf, 1)
    Hn.run_gsr(scene, cam, grads=grads, want_state=False)
    torch.cuda.synchronize()
    lib.gsr_stats_read(buf, 1)
    s = list(buf)
    for name, off in (("fwd", 0), ("bwd", 16)):
        it, ns, pre, full, okpx, batches, tail, inst, strips = s[off:off + 9]
        print(f"{name}: instances={inst} batches={batches} prefiltered={pre} zero_tail={tail} visited={it} "
              f"near_skip={ns} ({ns / max(it, 1):.1%}) full={full} strips={strips} ({strips / max(full, 1):.2f}/full) "
              f"ok_px={okpx} lane_eff={okpx / max(64 * strips, 1):.1%}")
    print(f"bwd batches with a lane whose replay starts inside the batch: {s[16 + 9]} of {s[16 + 5]}")
    print(f"fwd blended quadrants without a contributing pixel: {s[10]} of {s[8]}; bwd replayed strips without one: "
          f"{s[16 + 10]} of {s[16 + 8]}; bwd records whose replayed strips had none: {s[16 + 11]} of {s[16 + 3]}")


if __name__ == "__main__":
    main()
