"""Instances whose records the render kernels actually read, per BASELINE config (VERDICT r5
Next #5): early termination (forward.cu:343-359) stops the forward's list walk once every pixel
of the tile is done, and the backward replays only positions below the tile's deepest
contributor, so SURVEY s8(d)'s 52 B per instance x num_rendered overstates what a render
kernel can fetch (at C5 it implied 11.3 TB/s).  Counted by the GSR_STATS build (render.hip
stat 13: the records of every batch a wave processes).

Build:  make -C 3d_gaussian_magic_change-segment_3dgs_amd/csrc OUT=$PWD/build/diag/libgsr_stats.so \\
            HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -fvisibility=hidden -fno-slp-vectorize -DGSR_STATS" \
            SCHED_GAUSSIAN_BWD=      (the iterative-ilp scheduler crashes clang on the stats build)
Run:    python tools/fetched_instances.py [config ...] > profiles/round6_fetched_instances.json   (GPU)
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("GSR_LIBRARY", os.path.join(ROOT, "build", "diag", "libgsr_stats.so"))
sys.path[:0] = [ROOT, os.path.join(ROOT, "3d_gaussian_magic_change-segment_3dgs_amd"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402

from diff_gaussian_rasterization import _C  # noqa: E402
from gsr_tools.scene import config_scene_and_camera  # noqa: E402
import harness as Hn  # noqa: E402


def main(cfgs):
    lib = _C._lib
    lib.gsr_stats_read.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    buf = (ctypes.c_ulonglong * 32)()
    out = {"source": "GSR_STATS build of the round's sources (tools/fetched_instances.py)", "configs": {}}
    for cfg in cfgs:
        scene, cam = config_scene_and_camera(cfg)
        grads = Hn.upstream_grads(cam.height, cam.width)
        Hn.run_gsr(scene, cam, grads=grads, want_state=False)  # warm-up
        torch.cuda.synchronize()
        lib.gsr_stats_read(buf, 1)
        g = Hn.run_gsr(scene, cam, grads=grads, want_state=True)
        torch.cuda.synchronize()
        lib.gsr_stats_read(buf, 1)
        s = list(buf)
        out["configs"][cfg] = {"P": scene.P, "width": cam.width, "height": cam.height, "num_rendered": g["num_rendered"],
                               "fwd_fetched": s[13], "bwd_fetched": s[16 + 13], "fwd_batches": s[5],
                               "bwd_batches": s[16 + 5]}
        print(cfg, out["configs"][cfg], file=sys.stderr, flush=True)
        del g
        torch.cuda.empty_cache()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1:] or ["c1", "c2", "mt", "c3", "c5"])
