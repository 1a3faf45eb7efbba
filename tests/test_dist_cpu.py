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
    out_q.put((rank, b.numpy().copy(), bool(torch.equal(means2D_before, means2D_after))))
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
    for rank, b, m2d_untouched in res:
        np.testing.assert_allclose(b, ref, rtol=0, atol=1e-7)
        assert m2d_untouched, "per-view means2D gradients must not be reduced"


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
