"""A/B the fused Adam launch shapes (gsr_set_option adam_items / adam_nt / adam_grid)
at P = 1M, SH3 on the GPU; prints ms and GB/s per variant."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3d_gaussian_magic_change-segment_3dgs_amd"))
import torch  # noqa: E402
from diff_gaussian_rasterization import _C  # noqa: E402
from gsr_tools.scene import synthetic_scene  # noqa: E402
from gsr_tools import train_bench  # noqa: E402
from gsr_train import GaussianModel  # noqa: E402

P = int(os.environ.get("P", "1000000"))
sc = synthetic_scene(P, 3)
m = GaussianModel(3, device="cuda")
m.create_from_tensors(sc.means3D, sc.shs[:, :1], sc.shs[:, 1:], torch.logit(sc.opacities), torch.logit(sc.segments),
                      torch.log(sc.scales), sc.rotations)
m.training_setup(train_bench._TrainArgs)
g = torch.randn(m._spec.total, device="cuda") * 1e-3
B = train_bench.adam_bytes(P, 16)


def run():
    m._arena.grad = g
    m.optimizer.step()


for items in (1, 2, 4):
    for nt in (0, 1):
        for grid in (0, 2048, 8192):
            _C.set_option("adam_items", items)
            _C.set_option("adam_nt", nt)
            _C.set_option("adam_grid", grid)
            ms = min(train_bench._events_ms(run, 20) for _ in range(3))
            print(f"items={items} nt={nt} grid={grid:5d}: {ms:.4f} ms  {B / ms / 1e6:.0f} GB/s", flush=True)
