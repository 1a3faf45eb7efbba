"""CPU rehearsal of tests/test_gpu_exp_budget.py's oracle-side statements, per exp mode
(libm expf, +-1 ulp and +-2 ulp jitter of the shared exp): flipped pixels, the image and
weight-sum deviation on unflipped pixels, (ii) G vs L with the weight sums pinned, and the
unpinned deviation (G vs L from its own weight sums) whose maximum sets the test's guard.

    python tools/exp_budget_cpu.py [case ...] > profiles/round6_exp_modes.txt
"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "3d_gaussian_magic_change-segment_3dgs_amd")]

import harness as Hn  # noqa: E402
from contract_cases import case_scene  # noqa: E402
from oracle import oracle as O  # noqa: E402

CASES = ["c1", "sh3", "large", "c2", "mt", "c3", "c5"]
MODES = ["libm", "jit1", "jit2"]
KEYS = ("dmeans2D", "dopacity", "dmeans3D", "dsh", "dscales", "drot", "dsegments")
JITTER_SEED = 12345


def set_mode(mode):
    O.set_exp_libm(mode == "libm")
    O.set_exp_jitter(JITTER_SEED if mode.startswith("jit") else 0, ulps=int(mode[3:]) if mode.startswith("jit") else 1)


def normwise(a, b, k):
    a, b = np.asarray(a, np.float64).reshape(b.shape), b.astype(np.float64)
    if k == "dmeans2D":
        a, b = a[:, :2], b[:, :2]
    return np.abs(a - b) / max(float(np.abs(b).max()), 1e-30)


def main(cases, modes):
    worst = 0.0
    for name in cases:
        scene, cam = case_scene(name)
        H, W = cam.height, cam.width
        grads = Hn.upstream_grads(H, W)
        set_mode("none")
        own = O.run_scene(scene, cam)
        for mode in modes:
            t0 = time.time()
            set_mode(mode)
            try:
                lib = O.run_scene(scene, cam)
                flipped = (own.get("dhash") != lib.get("dhash")).reshape(H, W)
                keep = ~flipped
                km = torch.from_numpy(keep)[None]
                ups = [(grads[k] * km).contiguous().numpy() for k in ("color", "segment", "depth", "alpha")]
                img = 0.0
                for a, b in ((own.color, lib.color), (own.depth, lib.depth), (own.alpha, lib.alpha), (own.segment, lib.segment)):
                    e = np.abs(a.astype(np.float64) - b) / np.maximum(1.0, np.abs(b))
                    img = max(img, float(e[:, keep].max()))
                dw = float(np.abs(own.alpha[0].astype(np.float64) - lib.alpha[0])[keep].max())
                free = lib.backward(*ups)
                lib.set_weight_sums(own.alpha)
                pinned = lib.backward(*ups)
            finally:
                set_mode("none")
            G = own.backward(*ups)
            ii = {k: float(normwise(G[k], pinned[k], k).max()) for k in KEYS if k in G}
            un = {k: (float((normwise(G[k], free[k], k) > 1e-5).mean()), float(normwise(G[k], free[k], k).max()))
                  for k in KEYS if k in G}
            worst = max(worst, max(m for _, m in un.values()))
            print(f"{name} {mode}: flipped {int(flipped.sum())}/{flipped.size}; image {img:.1e}; dweight {dw:.1e}; "
                  f"(ii) max {max(ii.values()):.1e} (" + ", ".join(f"{k} {v:.1e}" for k, v in ii.items()) + "); unpinned " +
                  ", ".join(f"{k} {fr:.2%} (max {m:.1e})" for k, (fr, m) in un.items()) +
                  f"  [{time.time() - t0:.1f} s]", flush=True)
        del own
    print(f"# worst unpinned normwise deviation: {worst:.3e}")


if __name__ == "__main__":
    args = sys.argv[1:]
    main([a for a in args if a not in MODES] or CASES, [a for a in args if a in MODES] or MODES)
