"""distCUDA2 (submodules_local/simple-knn: ext.cpp / simple_knn.cu:181-220) on the
MI355X: mean squared distance of every point to its 3 nearest neighbours, used by
GaussianModel.create_from_pcd (scene/gaussian_model.py:143).  Kernels: csrc/knn.hip
(include/gsr_train.h gsr_dist_knn3)."""
import ctypes

import torch

from . import _C

_lib = _C._lib
_lib.gsr_knn_ws_bytes.restype = ctypes.c_size_t
_lib.gsr_knn_ws_bytes.argtypes = [ctypes.c_int]
_lib.gsr_dist_knn3.restype = ctypes.c_int
_lib.gsr_dist_knn3.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]


def distCUDA2(points):
    """points: float32 [P, 3] GPU tensor -> float32 [P] (reference name and contract)."""
    if points.dim() != 2 or points.shape[1] != 3:
        raise RuntimeError("distCUDA2: points must have shape (P, 3)")
    if points.device.type != "cuda":
        raise RuntimeError("distCUDA2: points must be a GPU tensor (the HIP path has no CPU fallback)")
    pts = points.detach().to(torch.float32).contiguous()
    P = int(pts.shape[0])
    out = torch.empty(P, dtype=torch.float32, device=pts.device)
    if P == 0:
        return out
    with torch.cuda.device(pts.device):
        ws = torch.empty(int(_lib.gsr_knn_ws_bytes(P)), dtype=torch.uint8, device=pts.device)
        _C._check(_lib.gsr_dist_knn3(P, pts.data_ptr(), out.data_ptr(), ws.data_ptr(), _C._stream(pts.device)))
    return out
