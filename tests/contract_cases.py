"""Scenes of the contraction / independent-exp studies: the BASELINE configs at full size
(view 0: the camera looks down the z axis, so view-space z is exact under any contraction)
plus rotated views of C2 and the metric scene (depth bits move) and two small parity scenes."""
import math

from gsr_tools.scene import config_scene_and_camera, orbit_camera, synthetic_scene


def case_scene(name):
    if name == "sh3":
        return synthetic_scene(20000, sh_degree=3, seed=3), orbit_camera(1, 333, 250, 300.0)
    if name == "large":  # 400 screen-filling Gaussians: every pixel sees ~100 of them
        return (synthetic_scene(400, sh_degree=2, seed=9, log_scale=math.log(0.4), log_scale_std=0.3),
                orbit_camera(3, 300, 200, 250.0))
    if name == "rot60k":
        return synthetic_scene(60000, sh_degree=3, seed=41), orbit_camera(3, 640, 360, 400.0)
    if "_v" in name:
        cfg, v = name.split("_v")
        return config_scene_and_camera(cfg, view_index=int(v))
    return config_scene_and_camera(name)
