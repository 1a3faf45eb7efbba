"""Per-config counts of integer outputs that move under the nvcc contraction model
(VERDICT r5 Next #1; tests/contract_study.py defines the statistics, oracle/gsr_oracle.cpp
"nvcc contraction model" the evaluation).  Oracle against oracle on the CPU: gsr's integer
outputs equal the uncontracted oracle's bit for bit (tests/test_gpu_full.py), so these are
also the counts by which gsr may differ from an nvcc build of the reference.

    python tools/contract_report.py [case ...] > profiles/round6_contract_counts.txt
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "3d_gaussian_magic_change-segment_3dgs_amd")]

import contract_study as CS  # noqa: E402
from contract_cases import case_scene  # noqa: E402
from oracle import oracle as O  # noqa: E402

CASES = ["c1", "sh3", "c2", "c2_v5", "mt", "mt_v3", "c3", "c5"]
MODES = [("pre", O.CT_PRE), ("pre-right", O.CT_PRE | O.CT_RIGHT), ("pre+blend", O.CT_PRE | O.CT_BLEND)]
COLS = ["visible", "moved", "radius_changed", "rect_changed", "tiles_touched_changed", "depth_bits_changed",
        "num_rendered", "d_num_rendered", "tiles_diff", "tiles_by_moved", "tiles_by_swap", "tiles_unexplained",
        "max_swap_ulps", "n_contrib_diff", "n_contrib_diff_outside_diff_tiles"]


def main(cases):
    print(f"# nvcc contraction model vs gsr's evaluation (oracle, {O.lib().oracle_num_threads()} threads)")
    print("case mode " + " ".join(COLS))
    for name in cases:
        scene, cam = case_scene(name)
        W, H = cam.width, cam.height
        t0 = time.time()
        O.set_contract(0)
        base = CS.from_oracle(O.run_scene(scene, cam), W, H)
        for label, mode in MODES:
            O.set_contract(mode)
            try:
                st = CS.compare(base, CS.from_oracle(O.run_scene(scene, cam), W, H), W, H)
            finally:
                O.set_contract(0)
            print(f"{name} {label} " + " ".join(str(st[c]) for c in COLS), flush=True)
        print(f"# {name}: P={scene.P} {W}x{H} pixels={W * H} ({time.time() - t0:.1f} s)", flush=True)


if __name__ == "__main__":
    main(sys.argv[1:] or CASES)
