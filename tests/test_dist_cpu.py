"""Multi-GPU path on the CPU: world size 2 over gloo, one view per rank, gradients
from the CPU oracle packed into gsr's gradient arena, one in-place all-reduce of
the parameter bucket (gsr_tools.dp, the same helper bench.py uses on RCCL).
The all-reduced bucket must equal the sum of the single-process per-view grads."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

P_TEST = 3000


def _per_view_grads(view):
    import sys
    sys.path[:0] = [ROOT, os.path.join(ROOT, "3d_gaussian_magic_change-segment_3dgs_amd"), os.path.join(ROOT, "tests")]
    import harness as Hn
    from oracle import oracle as O
    from gsr_tools.scene import synthetic_scene, orbit_camera
    scene = synthetic_scene(P_TEST, sh_degree=3, seed=31)
    cam = orbit_camera(view, 96, 64, 80.0, n_views=8)
    grads = Hn.upstream_grads(cam.height, cam.width, seed=1 + view)
    r = Hn.run_oracle(O, scene, cam, grads=grads)
    return r["grads"], scene.shs.shape[1]


def _worker(rank, world, port, out_q):
    import sys
    sys.path[:0] = [ROOT, os.path.join(ROOT, "3d_gaussian_magic_change-segment_3dgs_amd")]
    from gsr_tools import dp
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    g, M = _per_view_grads(rank)
    arena = dp.pack_arena(g, P_TEST, M)
    means2D_before = arena.narrow(0, dp.arena_layout(P_TEST, M)["dmeans2D"][0], 3 * P_TEST).clone()
    b = dp.allreduce_bucket(arena, P_TEST, M)
    means2D_after = arena.narrow(0, dp.arena_layout(P_TEST, M)["dmeans2D"][0], 3 * P_TEST)
    # the native exchange stays off on gloo / CPU tensors; dp.allreduce_async then issues
    # torch.distributed's all-reduce (the same sum, twice: the bucket is already reduced once)
    native = dp.init_native()
    b2 = dp.bucket(dp.pack_arena(g, P_TEST, M), P_TEST, M)
    dp.allreduce_async(b2).wait()
    out_q.put((rank, b.numpy().copy(), bool(torch.equal(means2D_before, means2D_after)), native,
               bool(torch.equal(b2, b))))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_view_parallel_allreduce_gloo_ws2():
    from gsr_tools import dp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # single-process reference: sum of the two views' bucket gradients
    ref = None
    for view in range(2):
        g, M = _per_view_grads(view)
        bk = dp.bucket(dp.pack_arena(g, P_TEST, M), P_TEST, M).numpy()
        ref = bk if ref is None else ref + bk
    for rank, b, m2d_untouched, native, async_equal in res:
        np.testing.assert_allclose(b, ref, rtol=0, atol=1e-7)
        assert m2d_untouched, "per-view means2D gradients must not be reduced"
        assert native is False, "the native RCCL exchange must stay off on gloo"
        assert async_equal, "dp.allreduce_async (torch.distributed fallback) must give the bucket all-reduce"


def _stats_worker(rank, world, port, out_q):
    import sys
    sys.path[:0] = [ROOT, os.path.join(ROOT, "3d_gaussian_magic_change-segment_3dgs_amd")]
    from gsr_tools import dp
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    g = torch.Generator().manual_seed(rank)
    accum, denom = torch.rand(100, 1, generator=g), torch.randint(0, 5, (100, 1), generator=g).float()
    radii = torch.randint(0, 50, (100,), generator=g).float()
    dp.reduce_densification_stats(accum, denom, radii)
    out_q.put((rank, accum.numpy().copy(), denom.numpy().copy(), radii.numpy().copy()))
    dist.barrier()
    dist.destroy_process_group()


def test_densification_stats_reduction_gloo_ws2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_stats_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = [None, None, None]
    for rank in range(2):
        g = torch.Generator().manual_seed(rank)
        a, d = torch.rand(100, 1, generator=g), torch.randint(0, 5, (100, 1), generator=g).float()
        r = torch.randint(0, 50, (100,), generator=g).float()
        ref = [a, d, r] if ref[0] is None else [ref[0] + a, ref[1] + d, torch.maximum(ref[2], r)]
    for rank, a, d, r in res:
        np.testing.assert_allclose(a, ref[0].numpy(), rtol=1e-6)
        assert np.array_equal(d, ref[1].numpy()) and np.array_equal(r, ref[2].numpy())


# ---- ShExchange: gathered dRGB rows + all-reduce of the non-SH blocks ----------
C0 = 0.28209479177387814  # auxiliary.h:21


def _sh_terms_f64(means3D, shs, deg, campos, drgb):
    """fp64 restatement (test-only) of one view's SH gradient terms: dsh = basis x dRGB
    (backward.cu:46-110) and the direction term of dmeans3D (the true derivative of
    dRGB . colour(dir(mean)), which the reference's hand formula computes)."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from test_oracle_autograd import sh_basis
    K = (deg + 1) ** 2
    m = means3D.double().clone().requires_grad_(True)
    d = m - campos.double()
    d = d / d.norm(dim=1, keepdim=True)
    bas = sh_basis(deg, d)  # [P, K]
    col = (bas[:, :, None] * shs.double()[:, :K, :]).sum(1)
    (dn,) = torch.autograd.grad((col * drgb.double()).sum(), m)
    dsh = torch.zeros(shs.shape, dtype=torch.float64)
    dsh[:, :K, :] = bas.detach()[:, :, None] * drgb.double()[:, None, :]
    return dsh, dn


def _sh_backward_f64(rows_all, V, means3D, sh, degree, dsh, dmeans3D):
    """Stand-in for _C.sh_backward on CPU tensors (reads the same row layout): dsh only --
    the direction term of dmeans3D is each rank's own, added before the exchange."""
    from diff_gaussian_rasterization._C import sh_rows_floats
    P = means3D.shape[0]
    ch = sh_rows_floats(P)
    cpos = ch - 64
    acc_sh = torch.zeros(sh.shape, dtype=torch.float64)
    for v in range(V):
        r = rows_all[v * ch:(v + 1) * ch]
        a, _ = _sh_terms_f64(means3D, sh, degree, r[cpos:cpos + 3], r[:3 * P].view(P, 3))
        acc_sh += a
    dsh.copy_(acc_sh.float())


def _sh_scene():
    import sys
    sys.path[:0] = [ROOT, os.path.join(ROOT, "3d_gaussian_magic_change-segment_3dgs_amd")]
    from gsr_tools.scene import synthetic_scene, orbit_camera
    return synthetic_scene(P_TEST, sh_degree=3, seed=31), [orbit_camera(v, 96, 64, 80.0, n_views=8) for v in range(2)]


def _sh_worker(rank, world, port, out_q):
    import sys
    sys.path[:0] = [ROOT, os.path.join(ROOT, "3d_gaussian_magic_change-segment_3dgs_amd")]
    from gsr_tools import dp
    from diff_gaussian_rasterization._C import sh_rows_floats
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    scene, cams = _sh_scene()
    g, M = _per_view_grads(rank)
    # deferred form of this view's gradients: dRGB rows + the complete dmeans3D (its SH
    # direction term included), dsh left as garbage (the exchange must overwrite all of it)
    drgb = torch.from_numpy(g["dsh"][:, 0, :]).float() / C0
    campos = cams[rank].camera_center.float()
    g = dict(g)
    g["dsh"] = np.full_like(g["dsh"], np.nan)
    arena = dp.pack_arena(g, P_TEST, M)
    lay = dp.arena_layout(P_TEST, M)
    dmeans3D = arena.narrow(0, lay["dmeans3D"][0], 3 * P_TEST).view(P_TEST, 3)
    dsh = arena.narrow(0, lay["dsh"][0], 3 * M * P_TEST).view(P_TEST, M, 3)
    ex = dp.ShExchange(sh_backward=_sh_backward_f64)
    rows = ex.sh_rows(1, P_TEST, torch.device("cpu"))
    rows.zero_()
    rows[:3 * P_TEST] = drgb.reshape(-1)
    rows[sh_rows_floats(P_TEST) - 64:sh_rows_floats(P_TEST) - 61] = campos
    ex.record(rows, 1, scene.means3D.float(), scene.shs.float(), 3, dsh, dmeans3D)
    ex.start().wait()
    out_q.put((rank, dp.bucket(arena, P_TEST, M).numpy().copy()))
    dist.barrier()
    dist.destroy_process_group()


def test_sh_exchange_gloo_ws2():
    """ShExchange's bucket equals the all-reduce of the complete per-view gradients."""
    from gsr_tools import dp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sh_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = None
    for view in range(2):
        g, M = _per_view_grads(view)
        bk = dp.bucket(dp.pack_arena(g, P_TEST, M), P_TEST, M).numpy()
        ref = bk if ref is None else ref + bk
    lay = dp.arena_layout(P_TEST, M)
    (r0, b0), (r1, b1) = sorted(res, key=lambda t: t[0])
    assert np.array_equal(b0, b1), "every rank must hold the same bits"
    for name in ("dmeans3D", "dsh", "dopacity", "dscales", "drot", "dsegments"):
        o, k = lay[name]
        a, r = b0[o:o + k * P_TEST], ref[o:o + k * P_TEST]
        err = np.abs(a.astype(np.float64) - r).max() / max(np.abs(r).max(), 1e-30)
        assert err < 2e-6, (name, err)


def test_exchange_choice():
    from gsr_tools import dp
    assert dp.choose_exchange(2, 1) == "sh" and dp.choose_exchange(8, 1) == "sh"
    assert dp.choose_exchange(8, 8) == "allreduce"
    c = dp.exchange_bytes(2, 1)
    assert c["allreduce"] / c["sh_exchange"] > 3.5


def test_exchange_time_model():
    """dp.exchange_cost / choose_exchange with P: the link time and the GPU-side work of both
    exchanges (the choice must include the SH rebuild's measured cost)."""
    from gsr_tools import dp
    P = 1_000_000
    c = dp.exchange_cost(8, 1, P, rebuild_us=55.0)
    assert c["sh_exchange"]["total_us"] < c["allreduce"]["total_us"]
    assert c["sh_exchange"]["rebuild_measured"] and c["sh_exchange"]["rebuild_us"] == 55.0
    assert dp.choose_exchange(2, 1, P=P, rebuild_us=40.0) == "sh"
    assert dp.choose_exchange(8, 8, P=P) == "allreduce"
    # a rebuild slower than the link time it saves flips the choice
    assert dp.choose_exchange(8, 1, P=P, rebuild_us=5000.0) == "allreduce"
    # with the compute time known, an exchange hidden behind the render costs only its GPU work
    h = dp.exchange_cost(8, 1, P, compute_us=930.0, rebuild_us=55.0)
    assert h["allreduce"]["total_us"] == round(930.0 + h["allreduce"]["gpu_us"], 2)
    assert dp.exchange_cost(1, 1, P)["allreduce"]["link_us"] == 0.0
    m = dp.rebuild_bytes(P, 8)
    assert m == (12 + 96 + 192) * P
