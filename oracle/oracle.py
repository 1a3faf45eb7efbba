"""ctypes front end of the CPU oracle (gsr_oracle.cpp).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py -- never by the product package.  See the header
of gsr_oracle.cpp for what the oracle restates and how it is pinned.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None


class OracleSettings(ctypes.Structure):
    _fields_ = [
        ("P", ctypes.c_int), ("D", ctypes.c_int), ("M", ctypes.c_int),
        ("W", ctypes.c_int), ("H", ctypes.c_int),
        ("tanfovx", ctypes.c_float), ("tanfovy", ctypes.c_float), ("scale_modifier", ctypes.c_float),
        ("prefiltered", ctypes.c_int),
        ("view", ctypes.c_float * 16), ("proj", ctypes.c_float * 16),
        ("campos", ctypes.c_float * 3), ("bg", ctypes.c_float * 3),
    ]


class OracleInputs(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in (
        "means3D", "shs", "colors_precomp", "segments", "opacities", "scales", "rotations", "cov3D_precomp")]


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.oracle_forward.restype = ctypes.c_void_p
        L.oracle_forward.argtypes = [ctypes.POINTER(OracleSettings), ctypes.POINTER(OracleInputs)] + [ctypes.c_void_p] * 5
        L.oracle_backward.restype = ctypes.c_int
        L.oracle_backward.argtypes = [ctypes.c_void_p, ctypes.POINTER(OracleInputs)] + [ctypes.c_void_p] * 13
        L.oracle_free.argtypes = [ctypes.c_void_p]
        L.oracle_num_rendered.argtypes = [ctypes.c_void_p]
        L.oracle_num_rendered.restype = ctypes.c_int
        L.oracle_get.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_void_p]
        L.oracle_get.restype = ctypes.c_long
        L.oracle_mark_visible.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        L.oracle_num_threads.restype = ctypes.c_int
        L.oracle_set_num_threads.argtypes = [ctypes.c_int]
        L.oracle_set_acc32.argtypes = [ctypes.c_int]
        L.oracle_set_exp_libm.argtypes = [ctypes.c_int]
        L.oracle_set_exp_jitter.argtypes = [ctypes.c_uint]
        L.oracle_set_exp_jitter_ulps.argtypes = [ctypes.c_int]
        L.oracle_set_contract.argtypes = [ctypes.c_int]
        L.oracle_get_contract.restype = ctypes.c_int
        L.oracle_set_weight_sums.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        L.oracle_expf.argtypes = [ctypes.c_float]
        L.oracle_expf.restype = ctypes.c_float
        L.oracle_dist_knn3.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
        _lib = L
    return _lib


def _f32(a):
    if a is None:
        return None
    if hasattr(a, "detach"):
        a = a.detach().cpu().numpy()
    a = np.ascontiguousarray(a, dtype=np.float32)
    return a if a.size else None


def _ptr(a):
    return None if a is None else a.ctypes.data


_FIELD_DTYPES = {
    "depths": np.float32, "means2D": np.float32, "cov3D": np.float32, "conic_opacity": np.float32,
    "rgb": np.float32, "clamped": np.uint8, "tiles_touched": np.uint32, "point_offsets": np.uint32,
    "keys": np.uint64, "point_list": np.uint32, "ranges": np.uint32, "n_contrib": np.uint32, "gabs": np.float32, "dhash": np.uint64,
}


def set_acc32(on):
    """True: accumulate per-pixel gradient terms in fp32 in one fixed order (emulates one
    run of the reference's atomicAdds); False (default): exact (fp64) sums."""
    lib().oracle_set_acc32(int(bool(on)))


def set_exp_libm(on):
    """True: blend with the C library's expf instead of gsr_expf (noise-floor studies)."""
    lib().oracle_set_exp_libm(int(bool(on)))


def set_exp_jitter(seed, ulps=1):
    """seed != 0: every blend exp moves by -ulps .. +ulps ulp (hash of seed, Gaussian, pixel),
    the same in forward and backward -- the reference algorithm under another exp of that
    accuracy around gsr_expf (CUDA's expf: 2 ulp); 0: off."""
    lib().oracle_set_exp_jitter_ulps(int(ulps))
    lib().oracle_set_exp_jitter(int(seed))


# nvcc contraction model (gsr_oracle.cpp "nvcc contraction model"): bit flags
CT_PRE, CT_BLEND, CT_RIGHT = 1, 2, 4


def set_contract(mode):
    """0 (default): every a*b+c rounded twice, as gsr evaluates it.  CT_PRE: the projection,
    ndc2Pix, cov3D, cov2D and the determinant / eigenvalue lines contracted into FMAs the way
    nvcc's default --fmad=true does (LLVM DAG-combine rule, left product of two fused;
    | CT_RIGHT: the right one); CT_BLEND: the blend's power and sums likewise."""
    lib().oracle_set_contract(int(mode))


def get_contract():
    return int(lib().oracle_get_contract())


def expf(x):
    """The blend exponential shared by the oracle and the HIP kernels (gsr_expf)."""
    return float(lib().oracle_expf(float(x)))


class OracleRun:
    """One forward call; keeps the reference's geometry/binning/image state for backward."""

    def __init__(self, settings, inputs):
        self._settings = settings
        self._inputs = inputs  # keep arrays alive
        s = settings
        self.P, self.W, self.H = s["P"], s["W"], s["H"]
        P, H, W = self.P, self.H, self.W
        self.color = np.zeros((3, H, W), np.float32)
        self.depth = np.zeros((1, H, W), np.float32)
        self.alpha = np.zeros((1, H, W), np.float32)
        self.segment = np.zeros((2, H, W), np.float32)
        self.radii = np.zeros((P,), np.int32)
        cs = OracleSettings()
        cs.P, cs.D, cs.M, cs.W, cs.H = P, s["D"], s["M"], W, H
        cs.tanfovx, cs.tanfovy, cs.scale_modifier = s["tanfovx"], s["tanfovy"], s["scale_modifier"]
        cs.prefiltered = int(s.get("prefiltered", False))
        cs.view[:] = [float(v) for v in np.asarray(s["viewmatrix"], np.float32).reshape(-1)]
        cs.proj[:] = [float(v) for v in np.asarray(s["projmatrix"], np.float32).reshape(-1)]
        cs.campos[:] = [float(v) for v in np.asarray(s["campos"], np.float32).reshape(-1)]
        cs.bg[:] = [float(v) for v in np.asarray(s["bg"], np.float32).reshape(-1)]
        self._cs = cs
        ci = OracleInputs()
        for k in ("means3D", "shs", "colors_precomp", "segments", "opacities", "scales", "rotations", "cov3D_precomp"):
            setattr(ci, k, _ptr(inputs.get(k)))
        self._ci = ci
        self.handle = lib().oracle_forward(ctypes.byref(cs), ctypes.byref(ci), _ptr(self.color), _ptr(self.depth),
                                           _ptr(self.alpha), _ptr(self.segment), _ptr(self.radii))
        self.num_rendered = lib().oracle_num_rendered(self.handle)

    def get(self, name):
        n = lib().oracle_get(self.handle, name.encode(), None)
        if n < 0:
            raise KeyError(name)
        out = np.zeros((n,), _FIELD_DTYPES[name])
        lib().oracle_get(self.handle, name.encode(), out.ctypes.data)
        return out

    def set_weight_sums(self, alpha):
        """The backward's T_final = 1 - alpha from another forward (oracle_set_weight_sums)."""
        a = np.ascontiguousarray(np.asarray(alpha, np.float32).reshape(-1))
        if a.size != self.W * self.H:
            raise ValueError("alpha must hold H*W values")
        lib().oracle_set_weight_sums(self.handle, a.ctypes.data)

    def backward(self, dL_dcolor, dL_dsegment, dL_ddepth, dL_dalpha):
        P, M = self.P, self._settings["M"]
        g = {
            "dmeans2D": np.zeros((P, 3), np.float32), "dcolors": np.zeros((P, 3), np.float32),
            "dopacity": np.zeros((P, 1), np.float32), "dmeans3D": np.zeros((P, 3), np.float32),
            "dcov3D": np.zeros((P, 6), np.float32), "dsh": np.zeros((P, max(M, 0), 3), np.float32),
            "dscales": np.zeros((P, 3), np.float32), "drot": np.zeros((P, 4), np.float32),
            "dsegments": np.zeros((P, 2), np.float32),
        }
        ups = [_f32(x) for x in (dL_dcolor, dL_dsegment, dL_ddepth, dL_dalpha)]
        rc = lib().oracle_backward(self.handle, ctypes.byref(self._ci), *[_ptr(u) for u in ups],
                                   *[_ptr(g[k]) for k in ("dmeans2D", "dcolors", "dopacity", "dmeans3D", "dcov3D",
                                                          "dsh", "dscales", "drot", "dsegments")])
        if rc != 0:
            raise RuntimeError("oracle backward failed")
        return g

    def __del__(self):
        try:
            if getattr(self, "handle", None):
                lib().oracle_free(self.handle)
                self.handle = None
        except Exception:
            pass


def settings_from_camera(cam, P, sh_degree, M, bg=(0.0, 0.0, 0.0), scale_modifier=1.0, prefiltered=False):
    return dict(P=P, D=sh_degree, M=M, W=cam.width, H=cam.height, tanfovx=cam.tanfovx, tanfovy=cam.tanfovy,
                scale_modifier=scale_modifier, prefiltered=prefiltered,
                viewmatrix=cam.world_view_transform.cpu().numpy(), projmatrix=cam.full_proj_transform.cpu().numpy(),
                campos=cam.camera_center.cpu().numpy(), bg=np.asarray(bg, np.float32))


def run_scene(scene, cam, bg=(0.0, 0.0, 0.0), scale_modifier=1.0, colors_precomp=None, cov3D_precomp=None,
              segments="scene", sh_degree=None):
    """Forward over a gsr_tools.scene.Scene with the reference's default argument path
    (shs + scales/rotations) unless precomputed colours / covariances are given."""
    inputs = {"means3D": _f32(scene.means3D), "opacities": _f32(scene.opacities)}
    if colors_precomp is None:
        inputs["shs"] = _f32(scene.shs)
        M = scene.shs.shape[1]
    else:
        inputs["colors_precomp"] = _f32(colors_precomp)
        M = 0
    if cov3D_precomp is None:
        inputs["scales"] = _f32(scene.scales)
        inputs["rotations"] = _f32(scene.rotations)
    else:
        inputs["cov3D_precomp"] = _f32(cov3D_precomp)
    inputs["segments"] = _f32(scene.segments) if isinstance(segments, str) else _f32(segments)
    D = scene.sh_degree if sh_degree is None else sh_degree
    st = settings_from_camera(cam, scene.P, D, M, bg=bg, scale_modifier=scale_modifier)
    return OracleRun(st, inputs)


def mark_visible(means3D, viewmatrix):
    m = _f32(means3D)
    P = 0 if m is None else m.shape[0]
    out = np.zeros((P,), np.uint8)
    v = np.ascontiguousarray(np.asarray(viewmatrix, np.float32))
    if P:
        lib().oracle_mark_visible(P, _ptr(m), _ptr(v), _ptr(out))
    return out.astype(bool)


def dist_knn3(points):
    """distCUDA2 restated (knn_oracle.cpp): mean squared distance to the 3 nearest
    neighbours of every point, float32 [P]."""
    pts = np.ascontiguousarray(points, dtype=np.float32).reshape(-1, 3)
    out = np.zeros(pts.shape[0], dtype=np.float32)
    if pts.shape[0]:
        lib().oracle_dist_knn3(pts.shape[0], pts.ctypes.data, out.ctypes.data)
    return out
