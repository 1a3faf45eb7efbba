"""A/B: run bench.py with every radix sort in look-back mode (gsr_set_option sort_lookback_max)."""
import sys, runpy, os
sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__))), os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "3d_gaussian_magic_change-segment_3dgs_amd")]
from diff_gaussian_rasterization import _C
_C.set_option("sort_lookback_max", 1 << 30)
sys.argv = ["bench.py", "--stages", "--no-cpu-baseline", "--no-train", "--steps", "30"]
runpy.run_path(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench.py"), run_name="__main__")
