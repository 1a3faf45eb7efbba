"""The multi-GPU path end to end with the real HIP kernels: spawned ranks, each rendering
its own view of the replicated scene through the drop-in GaussianRasterizer and running
libgsr's backward.  Two cases: two gloo ranks sharing cuda:0 (this pool gives a test one
GPU), and one RCCL rank ("nccl" backend, world size 1 -- RCCL refuses two ranks on one
device; the collectives, all_gather_into_tensor and the side-stream waits of the exchange
still run through RCCL on the GPU, as bench.py --gpus N issues them).  The exchanged
gradients must equal the sum of the ranks' single-view gradients (computed on each rank
with the same library, no exchange):

  * dp.allreduce_bucket(dp.arena_of(g)) -- the bucket all-reduce bench.py issues:
    bit-exact (a two-term fp32 sum is the same either way);
  * dp.ShExchange with torch.autograd.grad -- all-gather of the views' dRGB rows,
    all-reduce of the 13 non-SH floats, dsh rebuilt on every rank: normwise 1e-6
    (the rebuilt dsh sums basis x dRGB per view in another order);
  * dp.ShExchange with loss.backward() -- the parameters' .grad are the backward's
    arena views and are completed in place by h.wait();
and each rank's means2D gradient stays its own view's (densification statistics are
per view).  Reference: the single-GPU loop this shards, train.py:94-185, and the
gradient the reference accumulates per view (scene/gaussian_model.py:523-526).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P_TEST = 6000
NAMES = ("means3D", "shs", "opacities", "scales", "rotations", "segments")


def _setup(world):
    import sys
    sys.path[:0] = [ROOT, os.path.join(ROOT, "3d_gaussian_magic_change-segment_3dgs_amd"), os.path.join(ROOT, "tests")]
    import harness as Hn
    from gsr_tools.scene import synthetic_scene, orbit_camera
    scene = synthetic_scene(P_TEST, sh_degree=3, seed=61)
    views = []
    for v in range(max(world, 2)):
        cam = orbit_camera(v, 160, 120, 150.0, n_views=4)
        views.append((Hn.settings_for(cam, 3, "cuda"), {k: t.cuda() for k, t in Hn.upstream_grads(120, 160, seed=20 + v).items()}))
    leaves = {k: getattr(scene, k).detach().cuda().clone().requires_grad_(True) for k in NAMES}
    return leaves, views


def _render(leaves, view):
    from diff_gaussian_rasterization import GaussianRasterizer
    st, ups = view
    m2 = torch.zeros_like(leaves["means3D"], requires_grad=True)
    color, radii, depth, alpha, seg = GaussianRasterizer(st)(
        means3D=leaves["means3D"], means2D=m2, opacities=leaves["opacities"], shs=leaves["shs"],
        segments=leaves["segments"], scales=leaves["scales"], rotations=leaves["rotations"])
    outs = [color, depth, alpha, seg]
    gouts = [ups["color"], ups["depth"], ups["alpha"], ups["segment"]]
    return m2, outs, gouts


def _grad(leaves, view):
    m2, outs, gouts = _render(leaves, view)
    g = torch.autograd.grad(outs, [leaves[k] for k in NAMES] + [m2], gouts)
    return g


def _worker(rank, world, port, backend, out_q, native=False):
    import torch.distributed as dist
    try:
        torch.cuda.set_device(0)
        leaves, views = _setup(world)
        from diff_gaussian_rasterization import defer_sh_gradients
        from gsr_tools import dp
        kw = {"device_id": torch.device("cuda", 0)} if backend == "nccl" else {}
        dist.init_process_group(backend, init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world, **kw)
        P, M = P_TEST, leaves["shs"].shape[1]
        # reference: the ranks' single-view drop-in gradients, summed here (no exchange)
        gs = [_grad(leaves, views[v]) for v in range(world)]
        ref = {k: sum(g[i] for g in gs) for i, k in enumerate(NAMES)}
        ref_m2 = gs[rank][-1]
        res = {"backend": str(dist.get_backend())}
        # native: the exchanges below go through csrc/dp.hip (gsr_dp_*, libgsr's own RCCL
        # communicator) instead of torch.distributed's calls
        res["native"] = dp.init_native() if native else False

        # 1. bucket all-reduce over the backward's gradient arena
        g = _grad(leaves, views[rank])
        dp.allreduce_bucket(dp.arena_of(g[0]), P, M)
        torch.cuda.synchronize()
        res["allreduce"] = {k: float((a - ref[k]).abs().max()) for k, a in zip(NAMES, g)}
        res["allreduce_m2_equal"] = bool(torch.equal(g[-1], ref_m2))
        # 1b. the same through dp.allreduce_async (native when set up): bit-exact as well
        g = _grad(leaves, views[rank])
        h = dp.allreduce_async(dp.bucket(dp.arena_of(g[0]), P, M))
        h.wait()
        torch.cuda.synchronize()
        res["allreduce_async"] = {k: float((a - ref[k]).abs().max()) for k, a in zip(NAMES, g)}

        # 2. ShExchange around torch.autograd.grad
        ex = dp.ShExchange()
        with defer_sh_gradients(ex):
            g = _grad(leaves, views[rank])
        ex.start().wait()
        torch.cuda.synchronize()
        res["sh_grad"] = {k: float((a.double() - ref[k].double()).norm() / ref[k].double().norm())
                          for k, a in zip(NAMES, g)}
        res["sh_grad_m2_equal"] = bool(torch.equal(g[-1], ref_m2))

        # 3. ShExchange around loss.backward(): .grad completed in place by h.wait()
        for t in leaves.values():
            t.grad = None
        m2, outs, gouts = _render(leaves, views[rank])
        ex = dp.ShExchange(params=[leaves["opacities"]])
        with defer_sh_gradients(ex):
            torch.autograd.backward(outs, gouts)
        h = ex.start()
        h.wait()
        torch.cuda.synchronize()
        res["sh_backward"] = {k: float((leaves[k].grad.double() - ref[k].double()).norm() / ref[k].double().norm())
                              for k in NAMES}
        res["sh_backward_m2_equal"] = bool(torch.equal(m2.grad, ref_m2))

        # 4. misuse fails loudly: an existing .grad gets the unfinished blocks accumulated into it
        m2, outs, gouts = _render(leaves, views[rank])
        ex = dp.ShExchange()
        with defer_sh_gradients(ex):
            torch.autograd.backward(outs, gouts)
        try:
            ex.start().wait()
            res["misuse_raised"] = False
        except RuntimeError:
            res["misuse_raised"] = True
        bucket = dp.bucket(dp.arena_of(_grad(leaves, views[rank])[0]), P, M)
        res["bucket_floats"] = int(bucket.numel())
        dist.barrier()
        if res["native"]:
            dp.finalize_native()
        dist.destroy_process_group()
        out_q.put((rank, res, None))
    except Exception as e:  # report instead of hanging the parent on the queue
        import traceback
        out_q.put((rank, None, traceback.format_exc()))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("backend,world,native", [("gloo", 2, False), ("nccl", 1, False), ("nccl", 1, True)])
def test_ranks_real_backward_exchange(gpu_available, backend, world, native):
    """native=True: the exchanges issued by csrc/dp.hip over libgsr's own RCCL communicator
    (include/gsr.h gsr_dp_*), checked against the same sums."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, backend, q, native)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = [q.get(timeout=240) for _ in range(world)]
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for rank, r, err in res:
        assert err is None, f"rank {rank} failed:\n{err}"
    for rank, r, _ in res:
        assert r["backend"] == backend
        assert r["native"] == native, "native exchange not set up"
        for mode in ("allreduce", "allreduce_async"):
            for k, e in r[mode].items():
                assert e == 0.0, f"rank {rank} {mode} {k}: max |diff| {e:.3e}"
        for mode in ("sh_grad", "sh_backward"):
            for k, e in r[mode].items():
                assert e <= 1e-6, f"rank {rank} {mode} {k}: normwise error {e:.2e}"
        for mode in ("allreduce", "sh_grad", "sh_backward"):
            assert r[f"{mode}_m2_equal"], f"rank {rank} {mode}: means2D gradient must stay the rank's own view's"
        assert r["misuse_raised"], "accumulating into an existing .grad must raise"
        assert r["bucket_floats"] >= 61 * P_TEST
