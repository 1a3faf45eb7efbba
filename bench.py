#!/usr/bin/env python
"""bench.py -- forward+backward views/s of the gsr rasterizer (BASELINE.json metric).

One step = one view per rank through the drop-in boundary (N views
per iteration at N GPUs): _RasterizeGaussians.forward (incl. the reference's
num_rendered host sync) + .backward with fixed synthetic upstream gradients
(SURVEY.md s8d), on the synthetic metric scene (1M Gaussians, SH3, 2 segment
classes, 1920x1080) resident in HBM.  With N GPUs (torchrun, one process per GPU)
every rank renders its own view of the replicated scene and the parameter-gradient
bucket (61 f32 / Gaussian) is summed with one RCCL all-reduce per step, issued
asynchronously on RCCL's stream so that it overlaps the next step's render (the
metric excludes the optimizer step; every exchange completes inside the timed
region).  value = N * steps / max-over-ranks elapsed (weak scaling in views).
`batched` additionally times steps of 8 views per rank with one multi-view
backward and one exchange per step (--views-per-gpu sets the main mode).

Prints ONE JSON line on rank 0.  Extra objects:
  roofline     -- the dominant kernel (per-stage HIP events recorded by libgsr on
                  the stream it launches on): algorithmic bytes per launch / mean
                  launch time vs the 8 TB/s HBM peak and vs the streaming-copy rate
                  measured on the box (gsr_stream_copy); `traffic` = PMC-measured HBM
                  bytes per launch from profiles/ when a counter profile exists;
                  `cycles_per_valu_instr` = SIMD cycles per PMC VALU instruction (the
                  render kernels are bound by VALU issue and latency, not bytes).
  train_step   -- (N = 1) the s8f training step around the rasterizer: fused Adam
                  step / activation backward kernels vs the reference's torch
                  optimizer + activations on the same GPU (gsr_tools/train_bench.py).
  cpu_baseline -- the CPU oracle (C++ restatement of the reference kernels,
                  OpenMP) timed on this box's host cores on a bounded sample of the
                  same workload (whole views, rank 0, N = 1 only).
"""
import argparse
import gc
import contextlib
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "3d_gaussian_magic_change-segment_3dgs_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X spec (MI355X_MICROARCH.md, chip-level parameters)
SIMD_CLOCK_HZ = 2.4e9  # MI355X peak engine clock
# newest committed counter summary (tools/pmc.sh + tools/pmc_summary.py); its counter-derived
# fields are reported only when it was collected on the sources being benchmarked
PMC_SUMMARY = next((os.path.join(ROOT, "profiles", f) for f in
                    ("round6_pmc_summary.json", "round5_pmc_summary.json", "round4_pmc_summary.json", "round3_pmc_summary.json",
                     "round2_pmc_summary.json", "round1_pmc_summary.json")
                    if os.path.exists(os.path.join(ROOT, "profiles", f))), "")


def pmc_for_this_build():
    """(summary dict or None, provenance note)."""
    if not PMC_SUMMARY:
        return None, "no counter summary committed"
    d = json.load(open(PMC_SUMMARY))
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    try:
        from pmc_summary import sources_sha256
        cur = sources_sha256()
    finally:
        sys.path.pop(0)
    name = os.path.relpath(PMC_SUMMARY, ROOT)
    if d.get("sources_sha256") != cur:
        return None, f"{name} was collected on other sources (counter fields omitted)"
    return d, f"{name} (collected on these sources, sha256 {cur[:12]})"


# {lib}: the collective library the process group actually runs on (dist.get_backend():
# "nccl" is RCCL on ROCm, "gloo" the CPU rehearsal backend)
EXCHANGE_DESC = {
    "allreduce": "one {lib} all-reduce of the 61 f32/Gaussian grad bucket",
    "sh": "SH exchange: {lib} all-gather of each view's 3-float dRGB rows + all-reduce of the 13 non-SH "
          "f32/Gaussian, dsh rebuilt on every rank (gsr_tools.dp.ShExchange)",
    None: "",
}


def dist_info(dist):
    """What the process group really is: backend name, world size and, for nccl, the
    RCCL version torch was built against."""
    if dist is None:
        return {"backend": None, "world_size": 1, "collective_lib": None, "rccl_version": None}
    backend = str(dist.get_backend())
    ver = None
    if backend == "nccl":
        try:
            v = torch.cuda.nccl.version()
            ver = ".".join(str(x) for x in v) if isinstance(v, tuple) else str(v)
        except Exception:
            ver = None
    return {"backend": backend, "world_size": int(dist.get_world_size()),
            "collective_lib": "RCCL" if backend == "nccl" else backend, "rccl_version": ver}


def algorithmic_bytes(stage, P, I, HW, deg, views=1, T=0, written=None):
    """Bytes a stage must move per launch: SURVEY.md s8(d)'s per-unit figures
    (a7..a16) attributed to the gsr stage that does that work."""
    M = (deg + 1) ** 2
    if stage == "preprocess":      # a7: (119 + 12 M) B per Gaussian
        return (119 + 12 * M) * P
    if stage == "scan":            # a8
        return 8 * P
    if stage == "depth_sort":      # gsr-only stage: one read + write of (key, id) per Gaussian
        return 16 * P
    if stage == "duplicate":       # a9: 20 B per Gaussian + 12 B per instance
        return 20 * P + 12 * I
    if stage == "tile_sort":       # a10 + a11: one read + write of key + value per instance;
        return 24 * I + 8 * I      # its last pass also emits the tile ranges (identifyTileRanges)
    if stage == "ranges":          # heavy-first tile schedule (k_tile_order): ranges read + written, order
        return 20 * T
    if stage == "render_fwd":      # a12: 52 B per instance + 32 B per pixel
        return 52 * I + 32 * HW
    if stage == "render_bwd":      # a14 (per-instance + per-pixel part)
        return 52 * I + 36 * HW
    if stage == "gaussian_bwd":
        # the fused kernel's own minimal bytes (SURVEY's a14 + a15 + a16 figure,
        # (299 + 24 M) B, assumes separate launches that re-read the SH rows and pass dL_dmean3D /
        # dL_dcov3D through memory, and came out above the copy rate at 6M Gaussians).  Per
        # Gaussian and view: radii, tiles_touched, the in-block slot offset, opacity, means3D, rotation,
        # scale, clamp byte and the 36-B SH direction Jacobian read (93 B; round 5: the opacity copy
        # replaced the 32-B half record); dmeans2D, dopacity, dmeans3D,
        # dscales, drot, dsegments and the 12 M-float dsh row written (64 + 12 M B).  Per
        # instance: its written flag (1 B); per written record: 48 B (W, measured).
        W = written if written is not None else I
        return ((93 + 64 + 12 * M) * P + I + 48 * W) * views
    return 0


def view_bytes(P, I, HW, deg):
    """SURVEY.md s8d whole-view algorithmic bytes: (446 + 36 M) P + 148 I + 68 HW."""
    M = (deg + 1) ** 2
    return (446 + 36 * M) * P + 148 * I + 68 * HW


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(scene, cam, grads, budget_s=20.0):
    """The CPU oracle on whole views of the benchmark workload (fwd and bwd timed apart), on
    every CPU this process may run on (all host cores; `value`), and beside it
    on the pool's CPU share for one GPU (OMP_NUM_THREADS as the box sets it), plus BASELINE
    config C1 (10k Gaussians, SH0, 256x256) for scale."""
    from oracle import oracle as O
    from gsr_tools.scene import config_scene_and_camera
    O.build()
    up = [grads[k].numpy() for k in ("color", "segment", "depth", "alpha")]

    def views(sc, cm, ups, reps):
        tf = tb = 0.0
        for _ in range(reps):
            t0 = time.perf_counter()
            r = O.run_scene(sc, cm)
            t1 = time.perf_counter()
            r.backward(*ups)
            tb += time.perf_counter() - t1
            tf += t1 - t0
        return tf, tb

    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = None
    share = int(O.lib().oracle_num_threads())  # OMP_NUM_THREADS (the pool's share) or the runtime default

    def timed(threads, budget):
        O.lib().oracle_set_num_threads(threads)
        one = sum(views(scene, cam, up, 1))  # warm-up view (thread pool, page faults)
        reps = int(max(1, min(10, budget // max(one, 1e-3))))
        tf, tb = views(scene, cam, up, reps)
        return {"value": round(reps / (tf + tb), 4), "threads": threads, "fwd_ms_per_view": round(1e3 * tf / reps, 1),
                "bwd_ms_per_view": round(1e3 * tb / reps, 1), "views": reps}

    allc = timed(affinity or share, budget_s / 2)
    pool = timed(share, budget_s / 2) if affinity and share != affinity else None
    s1, c1 = config_scene_and_camera("c1")
    g1 = torch.Generator().manual_seed(1)
    up1 = [(torch.randn(c, c1.height, c1.width, generator=g1) * 1e-3).numpy() for c in (3, 2, 1, 1)]
    # C1 (10k Gaussians, 256x256) is too small for hundreds of threads: timed at every CPU, at the
    # pool's share and at 8 threads; `c1` reports the fastest (256 threads ran it slower
    # than one thread of this container)
    c1_runs = []
    for th in sorted({affinity or share, share, min(8, affinity or share)}):
        O.lib().oracle_set_num_threads(th)
        one = sum(views(s1, c1, up1, 1))
        r1 = int(max(3, min(20, 3.0 // max(one, 1e-3))))
        tf1, tb1 = views(s1, c1, up1, r1)
        c1_runs.append({"value": round(r1 / (tf1 + tb1), 2), "threads": th, "views": r1,
                        "fwd_ms_per_view": round(1e3 * tf1 / r1, 2), "bwd_ms_per_view": round(1e3 * tb1 / r1, 2)})
    c1_best = max(c1_runs, key=lambda r: r["value"])
    O.lib().oracle_set_num_threads(share)
    # the machine's CPUs are shared with other GPUs' jobs, so every CPU is not always the faster
    # setting: `value` is the faster of the two thread counts (the baseline is not handicapped)
    best = pool if pool and pool["value"] > allc["value"] else allc
    return {"value": best["value"], "unit": "views/s", "cores": best["threads"],
            "cores_note": (f"`value` = the faster of two timings: OpenMP threads = every CPU sched_getaffinity "
                           f"allows ({affinity} of the machine's os.cpu_count()={os.cpu_count()} logical CPUs, "
                           f"shared with other GPUs' jobs: 'all_cpus') and OMP_NUM_THREADS="
                           f"{os.environ.get('OMP_NUM_THREADS')} threads, the pool's CPU share for one GPU "
                           f"('pool_share')"),
            "affinity_cpus": affinity, "machine_cpus": os.cpu_count(),
            "kind": "port", "cpu_model": cpu_model(),
            "fwd_ms_per_view": best["fwd_ms_per_view"], "bwd_ms_per_view": best["bwd_ms_per_view"],
            "all_cpus": allc, "pool_share": pool,
            "c1": {"value": c1_best["value"], "unit": "views/s", "fwd_ms_per_view": c1_best["fwd_ms_per_view"],
                   "bwd_ms_per_view": c1_best["bwd_ms_per_view"], "threads": c1_best["threads"],
                   "by_threads": c1_runs,
                   "sample": f"{c1_best['views']} views of C1 (P={s1.P}, {c1.width}x{c1.height}, SH{s1.sh_degree}) "
                             f"per thread count after 1 warm-up view; value = the fastest thread count"},
            "sample": f"{allc['views']} whole fwd+bwd views of the benchmark workload (P={scene.P}, "
                      f"{cam.width}x{cam.height}, SH{scene.sh_degree}) after 1 warm-up view, per thread count; "
                      f"oracle/gsr_oracle.cpp built -O3 -fopenmp"}


def stream_copy_peak(lib, device, nbytes=1 << 30):
    """Achievable HBM rate on this box: gsr_stream_copy (float4, non-temporal loads and
    stores) of `nbytes`, best of 1/2/4 float4 per thread, read + write bytes / time."""
    src = torch.empty(nbytes // 4, dtype=torch.float32, device=device).fill_(1.0)
    dst = torch.empty_like(src)
    st = torch.cuda.current_stream(device).cuda_stream
    best = 0.0
    for u in (1, 2, 4):
        lib.gsr_stream_copy(src.data_ptr(), dst.data_ptr(), nbytes, u, st)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(10):
            lib.gsr_stream_copy(src.data_ptr(), dst.data_ptr(), nbytes, u, st)
        b.record()
        b.synchronize()
        best = max(best, 2 * nbytes * 10 / (a.elapsed_time(b) * 1e-3) / 1e9)
    del src, dst
    torch.cuda.empty_cache()
    return round(best, 1)


def exchange_trial(cand, timed, drain, rounds=2, steps=8, warm=3):
    """The measured exchange choice: cand maps an exchange name to its step function; after `warm`
    untimed steps of each, `rounds` alternating rounds of `steps` timed steps per exchange (timed
    returns the max over ranks), each exchange keeping its faster round.  One round each in a fixed
    order let the first candidate carry the warm-up (world 1: 0.95 vs 0.90 ms per step in the trial,
    0.849 vs 0.859 in steady state, profiles/round6_c_rccl_world1.txt).  Every value is the max over
    ranks, so every rank picks the same exchange.  Returns (chosen name, {name: seconds per step})."""
    trial = {kind: float("inf") for kind in cand}
    for fn in cand.values():
        for _ in range(warm):
            fn()
    drain()
    for _ in range(rounds):
        for kind, fn in cand.items():
            trial[kind] = min(trial[kind], timed(fn, steps) / steps)
    return min(trial, key=trial.get), trial


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="mt", help="gsr_tools.scene.CONFIGS key (default: the metric config)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=20.0, help="seconds of CPU-oracle work for cpu_baseline")
    ap.add_argument("--stages", action="store_true", help="print the per-stage table to stderr")
    ap.add_argument("--no-train", action="store_true", help="skip the train_step measurement (SURVEY.md s8f)")
    ap.add_argument("--views-per-gpu", type=int, default=1,
                    help="views per rank per step (1: the drop-in single-view API, BASELINE.md's N views per "
                         "iteration at N GPUs; >1: one multi-view backward and one all-reduce per step)")
    ap.add_argument("--batched-views", type=int, default=8,
                    help="also time steps of this many views per rank (reported under 'batched'; 1 = skip)")
    ap.add_argument("--exchange", choices=["auto", "allreduce", "sh"], default="auto",
                    help="N>1 gradient exchange: one all-reduce of the 61-float bucket, or the SH exchange "
                         "(all-gather of 3-float dRGB rows + all-reduce of 13 floats, gsr_tools.dp.ShExchange); "
                         "auto = the one with fewer bytes per link for the step's views per rank")
    args = ap.parse_args()
    from gsr_tools import launch
    if launch.needs_launch(args.gpus):
        # `python3 bench.py --gpus N` without torch.distributed.run: start the N ranks here
        # (children of this process, which never touches the GPU) and relay rank 0's line
        sys.exit(launch.spawn_ranks(args.gpus, [sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                    env=dict(os.environ, GSR_LAUNCHER="bench.py")))
    # The bench line is the only thing on stdout: native libraries (RCCL prints its version
    # banner at communicator set-up) write to file descriptor 1 directly, so fd 1 is pointed
    # at stderr for the run and the JSON line goes to the saved descriptor.
    sys.stdout.flush()
    json_fd = os.dup(1)
    os.dup2(2, 1)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world:
        print(f"[bench] --gpus {args.gpus} under a launcher with WORLD_SIZE={world}: running {world} rank(s)",
              file=sys.stderr)
    # one process per GPU; on a box with fewer GPUs than ranks (rehearsal runs with
    # GSR_DIST_BACKEND=gloo) ranks share devices round-robin
    dev_index = local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev_index)
    device = torch.device("cuda", dev_index)
    dist = None
    # GSR_DIST_FORCE=1 (under torch.distributed.run): a process group even at world size 1,
    # so a one-GPU box runs the exchange through RCCL exactly as the N-GPU bench issues it
    if world > 1 or os.environ.get("GSR_DIST_FORCE") == "1":
        import torch.distributed as dist
        from gsr_tools.launch import dist_timeout
        backend = os.environ.get("GSR_DIST_BACKEND", "nccl")  # nccl == RCCL over xGMI on ROCm
        # a bounded timeout (rendezvous and every collective; RCCL's watchdog aborts a stuck
        # collective after it): a hung rank fails the job instead of burning the driver's limit
        if backend == "nccl":
            dist.init_process_group(backend, device_id=device, timeout=dist_timeout())
        else:
            dist.init_process_group(backend, timeout=dist_timeout())
    native_dp = False

    from gsr_tools.scene import config_scene_and_camera
    from gsr_tools import dp
    if dist is not None:
        # the exchange's collectives from C over the library's own RCCL communicator (csrc/dp.hip;
        # GSR_NATIVE_DP=0: torch.distributed's calls)
        native_dp = dp.init_native()
    import diff_gaussian_rasterization as dgr
    from diff_gaussian_rasterization import _C

    B = max(1, min(args.views_per_gpu, 16))
    BB = max(1, min(args.batched_views, 16))  # the extra batched measurement
    NV = max(B, BB)
    n_views = max(8, world * NV)
    scene_cpu, cam_cpu = config_scene_and_camera(args.config, view_index=rank * NV, n_views=n_views)
    cams_cpu = [cam_cpu] + [config_scene_and_camera(args.config, view_index=rank * NV + j, n_views=n_views, P=1)[1]
                            for j in range(1, NV)]
    P, W, H, deg = scene_cpu.P, cam_cpu.width, cam_cpu.height, scene_cpu.sh_degree
    gen = torch.Generator().manual_seed(1)
    ups_cpu = {k: (torch.randn(c, H, W, generator=gen) * 1e-3) for k, c in
               (("color", 3), ("depth", 1), ("alpha", 1), ("segment", 2))}
    ups = {k: v.to(device) for k, v in ups_cpu.items()}
    leaf = lambda t: t.to(device).contiguous().requires_grad_(True)
    means3D, shs, opac = leaf(scene_cpu.means3D), leaf(scene_cpu.shs), leaf(scene_cpu.opacities)
    scales, rots, segs = leaf(scene_cpu.scales), leaf(scene_cpu.rotations), leaf(scene_cpu.segments)
    means2D = [torch.zeros_like(means3D, requires_grad=True) for _ in range(NV)]
    E = torch.empty(0, device=device)
    settings = [dgr.GaussianRasterizationSettings(
        image_height=H, image_width=W, tanfovx=c.tanfovx, tanfovy=c.tanfovy,
        bg=torch.zeros(3, device=device), scale_modifier=1.0, viewmatrix=c.world_view_transform.to(device),
        projmatrix=c.full_proj_transform.to(device), sh_degree=deg, campos=c.camera_center.to(device),
        prefiltered=False, debug=False) for c in cams_cpu]
    params = [means3D, shs, opac, scales, rots, segs]
    lay = _C.grad_arena_layout(P, shs.shape[1])
    state = {"I": 0}
    up_list = [ups["color"], ups["depth"], ups["alpha"], ups["segment"]]

    pending = []  # the exchange in flight: (work handle, gradients kept alive)
    # GSR_HOST_PROFILE=1: host seconds per step spent launching the view and the exchange
    HOST_PROFILE = os.environ.get("GSR_HOST_PROFILE") == "1"
    host_times = {"fwd+bwd": 0.0, "exchange": 0.0, "n": 0}

    def exchange_kind(nv, force=None):
        """The exchange for nv views per rank and its modelled cost (dp.exchange_cost), with the
        SH exchange's dsh rebuild timed on this GPU at the step's view count (world * nv rows)."""
        if dist is None:
            return None, None
        M = shs.shape[1]
        rb = dp.measure_rebuild_us(P, M, world * nv, device, degree=deg)
        model = dp.exchange_cost(world, nv, P, M, rebuild_us=rb)
        kind = force or (dp.choose_exchange(world, nv, M, P=P, rebuild_us=rb) if args.exchange == "auto"
                         else args.exchange)
        return kind, model

    def exchange(g, ex=None):
        # One exchange per step, on RCCL's stream (+ the SH completion on a side stream
        # for ShExchange): it runs while the next step renders (the metric excludes the
        # optimizer step, so no later work waits for it); at most one is in flight.
        if dist is None:
            return
        while pending:
            pending.pop()[0].wait()
        if ex is not None:
            h = ex.start()
        else:
            h = dp.allreduce_async(dp.bucket(dp.arena_of(g[0]), P, shs.shape[1]))
        pending.append((h, g))

    def drain():
        while pending:
            pending.pop()[0].wait()

    def make_step(nv, force=None):
        kind, model = exchange_kind(nv, force)

        def step():
            t0 = time.perf_counter()
            ex = dp.ShExchange() if kind == "sh" else None
            with dgr.defer_sh_gradients(ex) if ex is not None else contextlib.nullcontext():
                g = grads_of_views()
            t1 = time.perf_counter()
            exchange(g, ex)
            if HOST_PROFILE:
                host_times["fwd+bwd"] += t1 - t0
                host_times["exchange"] += time.perf_counter() - t1
                host_times["n"] += 1
            return g

        def grads_of_views():
            if nv == 1:
                # one view through the drop-in API (GaussianRasterizer's autograd function)
                color, radii, depth, alpha, segment = dgr.rasterize_gaussians(means3D, means2D[0], shs, E, segs,
                                                                              opac, scales, rots, E, settings[0])
                state["I"] = dgr._C.last_num_rendered(means3D.device)
                g = torch.autograd.grad([color, depth, alpha, segment], params + means2D[:1], up_list)
            else:
                # nv views: forward per view, one backward summing the parameter gradients
                # over the views (gsr_backward_multiview)
                outs = dgr.rasterize_gaussians_multiview(means3D, means2D[:nv], shs, E, segs, opac, scales, rots,
                                                         E, settings[:nv])
                state["I"] = sum(v[0] for v in outs[0][0].grad_fn.views) / nv
                g = torch.autograd.grad([t for o in outs for t in (o[0], o[2], o[3], o[4])],
                                        params + means2D[:nv], up_list * nv)
            return g
        step.exchange = kind
        step.exchange_model = model
        return step

    step = make_step(B)

    def written_records():
        """Instance slots the render backward stores a gradient record for, in one view (view 0)
        through the private bindings (outside any timed region): the per-record term of
        gaussian_bwd's algorithmic bytes."""
        rs = settings[0]
        out = _C.rasterize_gaussians(rs.bg, means3D, E, segs, opac, scales, rots, 1.0, E, rs.viewmatrix,
                                     rs.projmatrix, rs.tanfovx, rs.tanfovy, H, W, shs, deg, rs.campos, False, False)
        R, _, _, _, alpha, radii, geom, binning, img = out
        _C.rasterize_gaussians_backward(rs.bg, means3D, radii, E, segs, scales, rots, 1.0, E, rs.viewmatrix,
                                        rs.projmatrix, rs.tanfovx, rs.tanfovy, ups["color"], ups["segment"],
                                        ups["depth"], ups["alpha"], shs, deg, rs.campos, geom, R, binning, img,
                                        alpha, False)
        if R <= 0:
            return 0, 0
        wr = int(_C.debug_state("written", P, W, H, R, geom, binning, img).sum())
        # instances whose records the render backward reads: every position below its tile's deepest
        # contributor (front + back segments together), i.e. the sum of the per-tile max n_contrib
        # (equal to the GSR_STATS build's count, tools/fetched_instances.py)
        nct = _C.debug_state("n_contrib_tiles", P, W, H, R, geom, binning, img).view(-1, 256)
        return wr, int(nct.max(dim=1).values.to(torch.int64).sum())

    def timed(fn, k, per_step=None, stride=1, dom_mask=0):
        """k steps between a barrier + device sync on both sides; max over ranks.  Python's
        cyclic GC is paused (collected before the untimed stage pass that precedes this, not
        here: a collection while the GPU sits idle before the timed region let the clocks
        drop, and the first five timed steps ran 10-28% slow; a collection inside the loop
        stalls the host behind the per-view num_rendered sync).  per_step (a list) receives
        the mean step duration of every window of `stride` steps, from events recorded on the
        compute stream between the windows; the dominant stage's event bracket (dom_mask) is
        armed on the first step of each window.  An event costs the stream a few microseconds
        (the kernel trace showed ~5 us before the next kernel starts), so both are sampled
        once per window rather than every step."""
        nw = k // stride
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(nw + 1)] if per_step is not None else None
        if HOST_PROFILE:  # host times of the timed steps only
            host_times.update({"fwd+bwd": 0.0, "exchange": 0.0, "n": 0})
            if dp.HOST_TIMES is not None:
                dp.HOST_TIMES.clear()
        gc.disable()
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()
        t_start = time.perf_counter()
        if evs:
            evs[0].record()
        for i in range(k):
            if dom_mask:
                _C._lib.gsr_timing_enable(dom_mask if i % stride == 0 else 0)
            fn()
            if evs and (i + 1) % stride == 0 and (i + 1) // stride <= nw:
                evs[(i + 1) // stride].record()
        drain()
        torch.cuda.synchronize()
        gc.enable()
        if dist is not None:
            dist.barrier()
        el = time.perf_counter() - t_start
        if evs:
            per_step.extend(evs[w].elapsed_time(evs[w + 1]) / stride for w in range(nw))
        if dist is not None:
            t = torch.tensor([el], device=device, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        return el

    for _ in range(args.warmup):
        step()
    drain()
    torch.cuda.synchronize()
    if dist is not None and args.exchange == "auto" and step.exchange is not None:
        # The measured choice: the model (dp.exchange_cost) prices link bytes, HBM work and the
        # timed SH rebuild, but not the host's launch work per exchange, which can leave the GPU
        # idle between steps.  A few steps of each exchange (max over ranks) decide.
        modelled = step.exchange
        cand = {modelled: step}
        other = "allreduce" if modelled == "sh" else "sh"
        cand[other] = make_step(B, force=other)
        chosen, trial = exchange_trial(cand, timed, drain)
        step = cand[chosen]
        step.exchange_trial_ms = {k: round(1e3 * v, 4) for k, v in trial.items()}
        step.exchange_modelled = modelled
    nst = _C._lib.gsr_num_stages()
    import ctypes
    names = [_C._lib.gsr_stage_name(i).decode() for i in range(nst)]

    def collect():
        ms = (ctypes.c_double * nst)()
        cnt = (ctypes.c_longlong * nst)()
        _C._lib.gsr_timing_collect(ms, cnt)
        return ms, cnt

    collect()  # drop anything pending
    gc.collect()  # before the stage pass, so the GPU is busy right up to the timed region
    gc.disable()
    # Stage pass (untimed): every stage bracketed by events -> the stage table and the
    # dominant stage.  The brackets cost a few microseconds each, so the timed region
    # below records events around the dominant stage only.
    n_stage_steps = max(1, min(args.steps, 20))
    _C._lib.gsr_timing_enable(-1)
    for _ in range(n_stage_steps):
        step()
    drain()
    torch.cuda.synchronize()
    _C._lib.gsr_timing_enable(0)
    sms, scnt = collect()
    dom_i = max(range(nst), key=lambda i: sms[i]) if any(scnt) else 0
    step_ms = []
    stride = 4 if args.steps >= 8 else 1
    elapsed = timed(step, args.steps, step_ms, stride=stride, dom_mask=1 << dom_i)
    _C._lib.gsr_timing_enable(0)
    ms, cnt = collect()  # the dominant stage's launches inside the timed region (every 4th step)
    # The dominant kernel's launch time for `roofline`: right after the timed region, the same
    # steps again with libgsr's event bracket around EVERY launch of that stage (and no other
    # stage bracketed), so the mean is over every launch of the pass, not a sample.
    n_kpass = max(1, min(args.steps, 20))
    _C._lib.gsr_timing_enable(1 << dom_i)
    for _ in range(n_kpass):
        step()
    drain()
    torch.cuda.synchronize()
    _C._lib.gsr_timing_enable(0)
    kms, kcnt = collect()
    I, HW = int(state["I"]), W * H
    Wrec, Ibwd = written_records()  # gradient records stored (gaussian_bwd's bytes); instances the backward reads
    stages = {}
    for i in range(nst):
        if scnt[i]:
            avg = sms[i] / scnt[i]
            stages[names[i]] = {"avg_ms": round(avg, 4), "ms_per_step": round(sms[i] / n_stage_steps, 4),
                                "launches_per_step": scnt[i] / n_stage_steps,
                                "gbs": round(algorithmic_bytes(names[i], P, I, HW, deg, B, T=((W + 15) // 16) * ((H + 15) // 16),
                                                               written=Wrec)
                                             / (avg * 1e-3) / 1e9, 1)}
    dom = names[dom_i] if stages else None
    dinfo = dist_info(dist)
    value = world * B * args.steps / elapsed
    roof = None
    if dom and kcnt[dom_i]:
        avg_pass = kms[dom_i] / kcnt[dom_i]  # every launch of the dedicated pass after the timed region
        avg_window = ms[dom_i] / cnt[dom_i] if cnt[dom_i] else None  # sampled inside the timed region
        # the line's launch time is the one measured inside the timed region (every 4th step's
        # launch bracketed); the dedicated pass stands in only when the region had no sample
        avg_live = avg_window if avg_window else avg_pass
        achieved = round(algorithmic_bytes(dom, P, I, HW, deg, B, written=Wrec) / (avg_live * 1e-3) / 1e9, 1)
        traffic = cyc_per_valu = None
        pmc, pmc_note = pmc_for_this_build()
        if pmc is not None:
            try:
                pk = pmc.get("kernels", {}).get(dom, {})
                traffic = pk.get("hbm_bytes_per_launch")
                if pk.get("SQ_INSTS_VALU"):
                    # SIMD cycles per wave64 VALU instruction at the 2.4 GHz peak clock over the
                    # 1024 SIMDs: ~2.6-3.0 is the issue floor of plain f32 ops, 4.2-4.6 of compares,
                    # selects, min/max, shifts and SGPR-operand ops, ~8.5 of v_exp/v_rcp
                    # (tools/valu_mix_probe.hip, profiles/round2_valu_mix_probe.txt)
                    cyc_per_valu = round(SIMD_CLOCK_HZ * avg_live * 1e-3 * 1024 / pk["SQ_INSTS_VALU"], 3)
            except Exception:
                traffic = cyc_per_valu = None
        measured_peak = stream_copy_peak(_C._lib, device) if rank == 0 else None
        roof = {"bound": "hbm", "kernel": dom, "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                "measured_copy_peak": measured_peak,
                "frac_of_measured_peak": round(achieved / measured_peak, 4) if measured_peak else None,
                "algorithmic_bytes_per_launch": algorithmic_bytes(dom, P, I, HW, deg, B, written=Wrec),
                # SURVEY s8(d) counts every instance (52 B x num_rendered); early termination means the
                # render backward reads only the positions below each tile's deepest contributor
                # (Ibwd, measured here): the same kernel time against those bytes
                "fetched_instances": Ibwd if dom == "render_bwd" else None,
                "achieved_fetched": (round(algorithmic_bytes(dom, P, Ibwd, HW, deg, B) / (avg_live * 1e-3) / 1e9, 1)
                                     if dom == "render_bwd" else None),
                "frac_fetched": (round(algorithmic_bytes(dom, P, Ibwd, HW, deg, B) / (avg_live * 1e-3) / 1e9
                                       / HBM_PEAK_GBS, 4) if dom == "render_bwd" else None),
                "avg_launch_ms": round(avg_live, 4),
                "launches_timed": int(cnt[dom_i]) if avg_window else int(kcnt[dom_i]),
                "timing": (f"avg_launch_ms = mean of the hipEvent brackets libgsr records on its launch stream "
                           f"around the {dom} launch of every 4th step inside the timed region (only that stage "
                           f"bracketed there); avg_launch_ms_kernel_pass: the same bracket around every launch of "
                           f"{n_kpass} steps run right after the timed region; avg_launch_ms_stage_pass: every stage "
                           f"bracketed (untimed stage pass, inflated by the brackets); rocprofv3 --kernel-trace of "
                           f"this command, the metric phase's launches picked out by tools/ktrace_phases.py (the "
                           f"trace's kernel_stats average also holds the batched and train-step launches): "
                           f"profiles/round6_c_kernel_phases.txt"),
                "avg_launch_ms_timed_region": round(avg_window, 4) if avg_window else None,
                "avg_launch_ms_kernel_pass": round(avg_pass, 4),
                "avg_launch_ms_stage_pass": round(sms[dom_i] / scnt[dom_i], 4) if scnt[dom_i] else None,
                "valu_instr_per_launch": (pmc.get("kernels", {}).get(dom, {}).get("SQ_INSTS_VALU")
                                          if pmc is not None else None),
                "pmc_source": pmc_note,
                "cycles_per_valu_instr": cyc_per_valu,
                "whole_view_frac": round(view_bytes(P, I, HW, deg) * value / world / 1e9 / HBM_PEAK_GBS, 4)}
    out = {
        "metric": "forward+backward views/sec @1080p, 1M Gaussians, 1/2/4/8 MI355X",
        "value": round(value, 2), "unit": "views/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(1e3 * elapsed / args.steps, 4), "higher_is_better": True, "scaling": "weak",
        "step_ms": ({"mean": round(sum(step_ms) / len(step_ms), 4),
                     "median": round(sorted(step_ms)[len(step_ms) // 2], 4),
                     "p90": round(sorted(step_ms)[min(len(step_ms) - 1, int(0.9 * len(step_ms)))], 4),
                     "max_window": round(max(step_ms), 4),
                     # (first step index of the window, its per-step mean): windows, not single steps
                     "slowest_windows": [(i * stride, round(t, 3)) for t, i in
                                         sorted(((t, i) for i, t in enumerate(step_ms)), reverse=True)[:5]],
                     "window_steps": stride,
                     "source": f"hipEvents on the compute stream every {stride} steps; every statistic is over "
                               f"the per-step means of those {stride}-step windows, so a single slow step is "
                               f"diluted by its window (rank 0)"} if step_ms else None),
        "vs_baseline": None, "dtype": "f32", "data": "synthetic (SURVEY.md s8d generator, seed 0; upstream grads "
                                                    "N(0,1)*1e-3 seed 1)",
        "config": {"workload": f"{args.config}: P={P} Gaussians, SH{deg}, {W}x{H}, fwd+bwd per view; {B} view(s) per "
                               f"rank per step" + (" (per-view forward, one multi-view backward)" if B > 1 else
                                                   " through the drop-in GaussianRasterizer"), "P": P, "width": W, "height": H, "sh_degree": deg,
                   "num_classes": 2, "num_rendered": I, "written_records": Wrec, "bwd_fetched_instances": Ibwd, "global_batch": world * B, "views_per_step_per_gpu": B,
                   "parallelism": f"dp{world}" + ((" (views sharded; " +
                                                   EXCHANGE_DESC[step.exchange].format(lib=dinfo["collective_lib"]) +
                                                   " per step, overlapped with the next step's render)")
                                                  if dist is not None else ""),
                   "dist_backend": dinfo["backend"], "world_size": dinfo["world_size"],
                   "launcher": (os.environ.get("GSR_LAUNCHER") or
                                ("torch.distributed.run" if "TORCHELASTIC_RUN_ID" in os.environ else
                                 ("env" if "WORLD_SIZE" in os.environ else None))),
                   "rccl_version": dinfo["rccl_version"]},
        "roofline": roof,
        "stages": stages,
        "exchange": ({"chosen": step.exchange, "mode": args.exchange, "model_us": step.exchange_model,
                      "issued_by": ("gsr_dp_* over libgsr's own RCCL communicator (csrc/dp.hip)" if native_dp
                                    else "torch.distributed"),
                      "modelled_choice": getattr(step, "exchange_modelled", None),
                      "trial_ms_per_step": getattr(step, "exchange_trial_ms", None),
                      "model": "gsr_tools/dp.py exchange_cost: ring bytes over world-1 xGMI links at "
                               f"{dp.LINK_GBPS:g} GB/s x {dp.LINK_EFF:g} (assumed), HBM work at {dp.HBM_GBPS:g} GB/s, "
                               "the SH rebuild timed on this GPU"} if dist is not None else None),
    }
    if HOST_PROFILE and host_times["n"]:
        n = host_times["n"]
        out["host_us_per_step"] = {k: round(1e6 * v / n, 1) for k, v in host_times.items() if k != "n"}
        if dp.HOST_TIMES and dp.HOST_TIMES.get("n"):
            out["host_us_per_step"]["sh_exchange_start"] = {k: round(1e6 * v / dp.HOST_TIMES["n"], 1)
                                                            for k, v in dp.HOST_TIMES.items() if k != "n"}
    out["batched"] = None
    if BB > 1 and BB != B:
        # The same hot path with a batch of BB views per rank per step: per-view forward,
        # one multi-view backward and one exchange per step (bigger, fewer collectives
        # for point-to-point xGMI; SURVEY.md s8e / DESIGN.md s7).
        bstep = make_step(BB)
        # its own warm-up: the first batched steps grow the caching allocator's pools on both
        # streams and refill the binning-capacity guesses (BENCH_r04 timed 8 steps after 1
        # warm-up step: 1.014x; 16 after 3: 1.02x; the batched mode as the main measurement, 40
        # steps after 8: 1.062x, profiles/round5_bprof_kernel_stats.csv)
        for _ in range(max(8, args.warmup // 2)):
            bstep()
        drain()
        torch.cuda.synchronize()
        k = max(32, args.steps // BB)
        el_b = timed(bstep, k)
        # overlap of the two streams: every stage bracketed (untimed, 3 steps) -> the stage busy
        # time summed over both streams per step, against the wall time of the same steps
        collect()
        _C._lib.gsr_timing_enable(-1)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            bstep()
        drain()
        torch.cuda.synchronize()
        wall_b = (time.perf_counter() - t0) / 3
        _C._lib.gsr_timing_enable(0)
        bms, _ = collect()
        busy_b = sum(bms[i] for i in range(nst)) * 1e-3 / 3
        out["batched"] = {"views_per_step_per_gpu": BB, "global_batch": world * BB, "steps": k,
                          "value": round(world * BB * k / el_b, 2), "unit": "views/s",
                          "ms_per_step": round(1e3 * el_b / k, 4),
                          "exchange": bstep.exchange, "exchange_model_us": bstep.exchange_model,
                          "ratio_to_value": round(world * BB * k / el_b / value, 4),
                          "overlap": {"stage_busy_us_per_step": round(1e6 * busy_b, 1),
                                      "wall_us_per_step": round(1e6 * wall_b, 1),
                                      "busy_over_wall": round(busy_b / wall_b, 3) if wall_b > 0 else None,
                                      "note": "3 untimed steps with every stage bracketed by libgsr's events on "
                                              "the stream it launches on (the caller's and the side / auxiliary "
                                              "stream): busy time summed over both streams; > 1 = the streams "
                                              "overlapped"},
                          "note": "per-view forward + one gsr_backward_multiview over the batch + one exchange"}
    out["train_step"] = None
    if rank == 0 and world == 1 and not args.no_train:
        from gsr_tools import train_bench
        out["train_step"] = train_bench.measure(scene_cpu, cam_cpu, ups, device)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(scene_cpu, cam_cpu, ups_cpu, args.cpu_budget)
    else:
        out["cpu_baseline"] = None
    if rank == 0:
        if args.stages:
            for k, v in stages.items():
                print(f"{k:14s} {v['ms_per_step']:8.4f} ms/step  {v['gbs']:8.1f} GB/s", file=sys.stderr)
        sys.stdout.flush()
        os.write(json_fd, (json.dumps(out) + "\n").encode())
    if dist is not None:
        if native_dp:
            torch.cuda.synchronize()
            dp.finalize_native()  # libgsr's own RCCL communicator (csrc/dp.hip)
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
