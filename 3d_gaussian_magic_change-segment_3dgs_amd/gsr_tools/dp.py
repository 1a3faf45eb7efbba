"""View-parallel data parallelism for the rasterizer.

Each rank renders its own view of the replicated Gaussians; the exchange combines
the parameter-gradient bucket [dmeans3D | dsh | dopacity | dscales | drot |
dsegments] (61 f32 / Gaussian at SH3) over the ranks.  The backward writes every
gradient into one arena whose first `bucket` floats are exactly that bucket
(diff_gaussian_rasterization._C.grad_arena_layout), so an all-reduce runs in place
with no packing copy.  Backend "nccl" is RCCL over xGMI on ROCm; "gloo" is used for
the CPU tests.

Two exchanges give the same summed bucket:
  * allreduce_bucket: one all-reduce of all 61 floats;
  * ShExchange: the SH gradient of one view is basis(dir) x dRGB (backward.cu:46-110),
    so ranks all-gather each view's 3-float dRGB rows and rebuild the summed dsh
    (48 floats) locally; only the 13 non-SH floats are all-reduced.  Bytes per link
    at N ranks and B views per rank: allreduce 2(N-1)/N*244 B per Gaussian,
    ShExchange 2(N-1)/N*52 + (N-1)*B*12 B -- 3.8x less at N=2, 2.4x at N=8 (B=1).
    choose_exchange() picks the cheaper one.
"""
import ctypes
import os
import time

import torch
import torch.distributed as dist

# GSR_HOST_PROFILE=1: host seconds spent in ShExchange.start's phases (bench.py reports them)
HOST_TIMES = {} if os.environ.get("GSR_HOST_PROFILE") == "1" else None


def arena_layout(P, M):
    from diff_gaussian_rasterization._C import grad_arena_layout
    return grad_arena_layout(P, M)


def arena_of(grad_means3D):
    """The gradient arena behind the dmeans3D view returned by the backward."""
    base = grad_means3D._base
    if base is None or base.data_ptr() != grad_means3D.data_ptr():
        raise RuntimeError("gradient is not a view at the start of the gsr gradient arena")
    return base


def bucket(arena, P, M):
    return arena.narrow(0, 0, arena_layout(P, M)["bucket"][1])


def allreduce_bucket(arena, P, M, group=None):
    """Sum the parameter-gradient bucket over all ranks, in place; returns the bucket view."""
    b = bucket(arena, P, M)
    native_fence()
    dist.all_reduce(b, op=dist.ReduceOp.SUM, group=group)
    return b


def pack_arena(grads, P, M):
    """Build an arena from separate gradient tensors (CPU tests / foreign callers)."""
    lay = arena_layout(P, M)
    arena = torch.zeros(lay["total"][1], dtype=torch.float32)
    for name in ("dmeans3D", "dsh", "dopacity", "dscales", "drot", "dsegments", "dmeans2D", "dcolors", "dcov3D"):
        if name in grads and grads[name] is not None:
            o, k = lay[name]
            arena.narrow(0, o, k * P).copy_(torch.as_tensor(grads[name]).reshape(-1))
    return arena


def allreduce_model_grad(model, group=None):
    """Sum a gsr_train.GaussianModel's arena gradient over all ranks, in place.  The
    arena gradient has the bucket layout, so this is the same single collective."""
    g = model._arena.grad
    if g is not None:
        native_fence()
        dist.all_reduce(g, op=dist.ReduceOp.SUM, group=group)
    return g


def reduce_densification_stats(xyz_gradient_accum, denom, max_radii2D, group=None):
    """Combine per-rank densification statistics before densify_and_prune
    (SURVEY.md s8e): accumulated view-space gradient norms and view counts are
    summed, max_radii2D is max-reduced.  Each rank accumulated its own views'
    |dmeans2D| before any reduction, as the reference does per view."""
    both = torch.cat([xyz_gradient_accum.reshape(-1), denom.reshape(-1)])
    native_fence()
    dist.all_reduce(both, op=dist.ReduceOp.SUM, group=group)
    n = xyz_gradient_accum.numel()
    xyz_gradient_accum.copy_(both[:n].view_as(xyz_gradient_accum))
    denom.copy_(both[n:].view_as(denom))
    dist.all_reduce(max_radii2D, op=dist.ReduceOp.MAX, group=group)


def exchange_bytes(world, views_per_rank, M=16):
    """Bytes per Gaussian that each rank sends (ring model) for both exchanges."""
    n, b = int(world), int(views_per_rank)
    full = 4 * (13 + 3 * M)
    return {"allreduce": 2 * (n - 1) / n * full,
            "sh_exchange": 2 * (n - 1) / n * 4 * 13 + (n - 1) * b * 12}


# Time model of the exchange (us per step).  Link: xGMI, 153 GB/s per link and direction
# (MI355X spec), of which RCCL is assumed to reach LINK_EFF; an 8-GPU node is fully
# connected, so a rank's ring traffic can spread over its world - 1 peer links.  Both
# numbers are assumptions until the driver's SCALE run measures them; they scale both
# exchanges alike, so they matter only against the GPU-side costs below.
LINK_GBPS = 153.0
LINK_EFF = 0.7
HBM_GBPS = 5000.0  # a streaming kernel's rate on MI355X (measured copy: 6.5 TB/s)


def rebuild_bytes(P, views, M=16):
    """HBM bytes of the SH exchange's dsh rebuild (gsr_sh_backward, k_sh_dsh): means3D,
    each view's dRGB row, the dsh rows written."""
    return (12 + 12 * int(views) + 12 * int(M)) * int(P)


def exchange_cost(world, views_per_rank, P, M=16, compute_us=None, rebuild_us=None, link_gbps=None,
                  hbm_gbps=HBM_GBPS):
    """Modelled cost of both exchanges per step.  link_us: the ring traffic over the peer
    links; gpu_us: HBM work the exchange adds on each GPU (RCCL's reductions ~3 passes over
    the reduced bytes, the all-gathered rows, and for the SH exchange the dsh rebuild --
    `rebuild_us` when it was measured, else modelled from rebuild_bytes).  The exchange of
    step k overlaps step k+1's render, so a step costs max(compute + gpu, link) when the
    compute time is known, gpu + link otherwise."""
    n, b, P = int(world), int(views_per_rank), int(P)
    if n <= 1:  # nothing crosses a link; the SH exchange still rebuilds dsh
        rb = rebuild_us if rebuild_us is not None else rebuild_bytes(P, b, M) / (hbm_gbps * 1e3)
        return {"allreduce": {"link_us": 0.0, "gpu_us": 0.0, "total_us": compute_us or 0.0},
                "sh_exchange": {"link_us": 0.0, "gpu_us": round(rb, 2), "total_us": round((compute_us or 0.0) + rb, 2),
                                "rebuild_us": round(rb, 2), "rebuild_measured": rebuild_us is not None}}
    rate = (link_gbps or LINK_GBPS * LINK_EFF) * (n - 1) * 1e3  # bytes per us
    by = exchange_bytes(n, b, M)
    hbm = hbm_gbps * 1e3
    red = 3 * (n - 1) / n
    modelled_rebuild = rebuild_bytes(P, n * b, M) / hbm
    gpu = {"allreduce": red * 4 * (13 + 3 * M) * P / hbm,
           "sh_exchange": (red * 4 * 13 * P + 12 * n * b * P) / hbm +
                          (rebuild_us if rebuild_us is not None else modelled_rebuild)}
    out = {}
    for k in ("allreduce", "sh_exchange"):
        link_us = by[k] * P / rate
        tot = max(compute_us + gpu[k], link_us) if compute_us else gpu[k] + link_us
        out[k] = {"link_us": round(link_us, 2), "gpu_us": round(gpu[k], 2), "total_us": round(tot, 2)}
    out["sh_exchange"]["rebuild_us"] = round(rebuild_us if rebuild_us is not None else modelled_rebuild, 2)
    out["sh_exchange"]["rebuild_measured"] = rebuild_us is not None
    return out


def choose_exchange(world, views_per_rank, M=16, P=None, compute_us=None, rebuild_us=None):
    """"sh" or "allreduce".  With P: the cheaper modelled step (exchange_cost, including the
    measured or modelled dsh rebuild); without: the fewer link bytes."""
    if P is None:
        c = exchange_bytes(world, views_per_rank, M)
        return "sh" if c["sh_exchange"] < c["allreduce"] else "allreduce"
    c = exchange_cost(world, views_per_rank, P, M, compute_us=compute_us, rebuild_us=rebuild_us)
    return "sh" if c["sh_exchange"]["total_us"] < c["allreduce"]["total_us"] else "allreduce"


def measure_rebuild_us(P, M, views, device, degree=3, reps=5):
    """Time gsr_sh_backward (the SH exchange's dsh rebuild) for `views` views' rows of P
    Gaussians on this GPU: the median of `reps` launches, in us."""
    from diff_gaussian_rasterization import _C
    g = torch.Generator(device="cpu").manual_seed(0)
    means3D = torch.randn(P, 3, generator=g).to(device)
    rows = torch.randn(int(views) * _C.sh_rows_floats(P), generator=g).to(device) * 1e-3
    dsh = torch.empty(P, M, 3, device=device)
    sh = torch.empty(P, M, 3, device=device)
    ts = []
    for _ in range(reps + 1):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        _C.sh_backward(rows, int(views), means3D, sh, degree, dsh, None)
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    ts = sorted(ts[1:])
    return ts[len(ts) // 2]


# ---- native exchange (csrc/dp.hip, include/gsr.h gsr_dp_*): the same collectives issued from C
# over the library's own RCCL communicator.  torch.distributed's call path costs 25-35 us of host
# time per collective; at one view per rank the SH exchange's start then took 130-170 us of a
# 0.9-ms step and the host bounded the step (profiles/round4_c_rccl_world1_sh.json).
_UNSET = object()
_NATIVE = {"group": _UNSET, "last": None}  # the group init_native set up; the last ticket issued


def native_fence():
    """Order the current stream after the last native exchange before a torch.distributed
    collective is issued.  torch's collectives run on the process group's stream, which waits
    for the current stream, so with this fence no collective of torch's communicator can run
    beside one of libgsr's: the two communicators' collectives execute in one order on every
    rank (the native call itself orders its stream after the current stream, csrc/dp.hip
    dp_begin).  No-op when the native path is off."""
    t = _NATIVE["last"]
    if t is None or _NATIVE["group"] is _UNSET:
        return
    L = _lib()._lib
    if torch.cuda.is_initialized() and L.gsr_dp_world() > 0:
        _lib()._check(L.gsr_dp_wait(t, torch.cuda.current_stream().cuda_stream))


def _lib():
    from diff_gaussian_rasterization import _C
    return _C


def init_native(group=None):
    """Set up the native RCCL exchange beside torch.distributed's group `group` (the default group
    when None): group rank 0's unique id is broadcast over the group, every rank joins.  Collective:
    every rank of the group calls it.  Returns True when the native path is active; False (the
    torch.distributed path stays) with GSR_NATIVE_DP=0, a non-nccl backend or a library without
    it."""
    C = _lib()
    L = C._lib
    if (os.environ.get("GSR_NATIVE_DP", "1") == "0" or not hasattr(L, "gsr_dp_init")
            or dist.get_backend(group) != "nccl"):
        return False
    if L.gsr_dp_world() > 0:
        return _NATIVE["group"] is group
    if dist.get_world_size(group) > 1 and os.environ.get("GSR_NATIVE_DP") is None:
        # world > 1: the native path is opt-in (GSR_NATIVE_DP=1) until a multi-GPU run has
        # exercised it; bench.py and the trainer use torch.distributed's collectives otherwise
        return False
    n = int(L.gsr_dp_unique_id_bytes())
    uid = ctypes.create_string_buffer(n)
    if dist.get_rank(group) == 0:
        C._check(L.gsr_dp_get_unique_id(uid))
    obj = [uid.raw]
    dist.broadcast_object_list(obj, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
    uid = ctypes.create_string_buffer(obj[0], n)
    C._check(L.gsr_dp_init(uid, dist.get_world_size(group), dist.get_rank(group)))
    _NATIVE["group"] = group
    return True


def native_for(group, t):
    """The native exchange serves this group and CUDA tensor."""
    if not (t.is_cuda and _NATIVE["group"] is group):
        return False
    L = _lib()._lib
    return hasattr(L, "gsr_dp_world") and L.gsr_dp_world() == dist.get_world_size(group)


def finalize_native():
    C = _lib()
    if hasattr(C._lib, "gsr_dp_finalize"):
        C._check(C._lib.gsr_dp_finalize())
    _NATIVE["group"] = _UNSET
    _NATIVE["last"] = None


class _NativeTicket:
    """wait() orders the current stream after a native exchange (gsr_dp_wait); keeps the
    tensors the exchange reads or writes alive until then."""

    def __init__(self, ticket, keep):
        self.ticket, self.keep = ticket, keep

    def wait(self):
        if self.ticket is not None:
            C = _lib()
            C._check(C._lib.gsr_dp_wait(self.ticket, torch.cuda.current_stream().cuda_stream))
        self.ticket, self.keep = None, None

    def __del__(self):
        if getattr(self, "ticket", None) is not None:
            try:
                self.wait()
            except Exception:
                pass


def allreduce_async(t, group=None):
    """In-place sum of the fp32 tensor t over the group, asynchronous: a handle whose wait()
    orders the current stream after it (native when init_native set it up, else
    torch.distributed)."""
    if native_for(group, t) and t.dtype == torch.float32 and t.is_contiguous():
        C = _lib()
        tk = C._lib.gsr_dp_allreduce(t.data_ptr(), t.numel(), torch.cuda.current_stream(t.device).cuda_stream)
        if tk < 0:
            raise RuntimeError(C._lib.gsr_last_error().decode())
        _NATIVE["last"] = tk
        return _NativeTicket(tk, (t,))
    native_fence()
    return dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group, async_op=True)


def _all_gather_flat(out, inp, group, async_op):
    """all_gather into one flat buffer (RCCL: all_gather_into_tensor; gloo: list form)."""
    if dist.get_backend(group) == "nccl":
        return dist.all_gather_into_tensor(out, inp, group=group, async_op=async_op)
    world = dist.get_world_size(group)
    return dist.all_gather(list(out.view(world, -1).unbind(0)), inp, group=group, async_op=async_op)


class ShExchange:
    """View-parallel gradient exchange with the SH gradient rebuilt from gathered
    dRGB rows (include/gsr.h gsr_sh_backward).  Usage, once per step:

        ex = ShExchange(group)
        with diff_gaussian_rasterization.defer_sh_gradients(ex):
            grads = torch.autograd.grad(...)        # or loss.backward()
        h = ex.start()       # collectives + SH completion, asynchronous
        ...                  # more work (e.g. the next view's render)
        h.wait()             # the bucket now equals allreduce_bucket's result

    Nothing may read the deferred dsh / dmeans3D before h.wait().  On GPU tensors the
    collectives run on the process group's stream and the SH completion on a side
    stream that waits for them; h.wait() orders the caller's stream after it.

    With loss.backward() the parameters' .grad must be the backward's gradient views
    themselves (autograd hands them over without a copy when .grad is None, i.e. after
    zero_grad(set_to_none=True), and when the rasterizer inputs are the leaves or
    gsr_train's arena parameters): the exchange completes them in place.  The recorder
    therefore keeps no reference to the returned gradient tensors (a reference would
    make autograd clone them before they are complete).  If autograd did copy or
    accumulate into a leaf's existing .grad (a .grad that was not None, or a graph
    between the leaf and the rasterizer that reshapes the gradient), h.wait() raises
    instead of leaving a gradient computed from unfinished memory.
    `sh_backward` replaces _C.sh_backward (CPU tests pass the oracle's)."""

    def __init__(self, group=None, sh_backward=None, params=()):
        """params: further leaf tensors whose .grad comes from the exchanged bucket
        (e.g. the opacity leaf, which the backward does not see) -- checked at wait()
        like the rasterizer inputs."""
        self.group = group
        self.entries = []
        self._sh_backward = sh_backward
        self._params = tuple(params)

    # -- called by the deferred backward (diff_gaussian_rasterization._backward_views)
    def sh_rows(self, B, P, device):
        from diff_gaussian_rasterization._C import sh_rows_floats
        return torch.empty(B * sh_rows_floats(P), dtype=torch.float32, device=device)

    def record(self, rows, B, means3D, sh, degree, dsh, dmeans3D, inputs=()):
        arena = arena_of(dmeans3D)
        P, M = int(means3D.size(0)), int(sh.size(1))
        lay = arena_layout(P, M)
        if dsh.data_ptr() != arena.data_ptr() + 4 * lay["dsh"][0]:
            raise RuntimeError("deferred dsh is not the dsh block of the gradient arena")
        # leaves whose .grad autograd fills after this backward returns: remember what
        # .grad was, to detect at wait() a copy / accumulation of the unfinished blocks
        watch = []
        seen = set()
        for t in (means3D, sh) + tuple(inputs) + self._params:
            if isinstance(t, torch.Tensor) and t.is_leaf and t.requires_grad and id(t) not in seen:
                seen.add(id(t))
                gr = t.grad
                watch.append((t, gr, None if gr is None else gr._version))
        m3 = means3D.detach()
        if m3.is_cuda and (m3.dtype != torch.float32 or not m3.is_contiguous() or rows.device != m3.device or
                           rows.dtype != torch.float32 or not rows.is_contiguous()):
            raise RuntimeError("ShExchange: means3D and the rows must be contiguous float32 tensors on one device")
        self.entries.append(dict(rows=rows, B=B, means3D=m3, sh=sh.detach(), degree=int(degree),
                                 arena=arena, P=P, M=M, watch=watch))

    def start(self):
        if not self.entries:
            raise RuntimeError("ShExchange.start(): no deferred backward was recorded (run the backward inside "
                               "diff_gaussian_rasterization.defer_sh_gradients(exchange))")
        entries, self.entries = self.entries, []
        return _ShExchangeHandle([self._start_one(e) for e in entries])

    def _start_one(self, e):
        t0 = time.perf_counter() if HOST_TIMES is not None else 0.0
        P, M = e["P"], e["M"]
        lay = arena_layout(P, M)
        arena, rows = e["arena"], e["rows"]
        world = dist.get_world_size(self.group)
        xyz = arena.narrow(0, lay["dmeans3D"][0], 3 * P)
        o_rest = lay["dopacity"][0]
        rest = arena.narrow(0, o_rest, lay["bucket"][1] - o_rest)
        rows_all = torch.empty(world * rows.numel(), dtype=rows.dtype, device=rows.device)
        cuda = rows.is_cuda
        if self._sh_backward is None and native_for(self.group, rows):
            # one C call: the collectives as one RCCL group + the dsh rebuild, on the library's stream
            C = _lib()
            tk = C._lib.gsr_dp_sh_exchange(P, e["degree"], M, C.NUM_CLASS, e["means3D"].data_ptr(), e["B"],
                                           arena.data_ptr(), rows.data_ptr(), rows_all.data_ptr(),
                                           torch.cuda.current_stream(rows.device).cuda_stream)
            if tk < 0:
                raise RuntimeError(C._lib.gsr_last_error().decode())
            _NATIVE["last"] = tk
            if HOST_TIMES is not None:
                HOST_TIMES["native"] = HOST_TIMES.get("native", 0.0) + time.perf_counter() - t0
                HOST_TIMES["n"] = HOST_TIMES.get("n", 0) + 1
            return (_NativeTicket(tk, (arena, rows, rows_all, e["means3D"], e["sh"])), None, e)
        # (torch's _coalescing_manager around these three left rows_all unfilled on RCCL at
        # world size 1 -- tests/test_gpu_dist.py caught it: three calls)
        native_fence()
        t1 = time.perf_counter() if HOST_TIMES is not None else 0.0
        works = [dist.all_reduce(xyz, op=dist.ReduceOp.SUM, group=self.group, async_op=True),
                 dist.all_reduce(rest, op=dist.ReduceOp.SUM, group=self.group, async_op=True),
                 _all_gather_flat(rows_all, rows, self.group, True)]
        t2 = time.perf_counter() if HOST_TIMES is not None else 0.0
        V = world * e["B"]
        fn = self._sh_backward
        keep = (arena, rows, rows_all, e["means3D"], e["sh"])
        if not cuda:
            for w in works:
                w.wait()
            dsh = arena.narrow(0, lay["dsh"][0], 3 * M * P).view(P, M, 3)
            dmeans3D = arena.narrow(0, lay["dmeans3D"][0], 3 * P).view(P, 3)
            fn(rows_all, V, e["means3D"], e["sh"], e["degree"], dsh, dmeans3D)
            return (None, keep, e)
        side = _side_stream(rows.device)
        side.wait_stream(torch.cuda.current_stream(rows.device))
        with torch.cuda.stream(side):
            for w in works:
                w.wait()  # stream-side wait on the collective
            if fn is None:
                # gsr_sh_backward straight through ctypes: the tensors were checked when the
                # backward made them (record), and dsh is the arena's dsh block
                from diff_gaussian_rasterization import _C
                _C._check(_C._lib.gsr_sh_backward(V, P, e["degree"], M, None, e["means3D"].data_ptr(),
                                                  rows_all.data_ptr(), arena.data_ptr() + 4 * lay["dsh"][0], None,
                                                  side.cuda_stream))
            else:
                dsh = arena.narrow(0, lay["dsh"][0], 3 * M * P).view(P, M, 3)
                dmeans3D = arena.narrow(0, lay["dmeans3D"][0], 3 * P).view(P, 3)
                fn(rows_all, V, e["means3D"], e["sh"], e["degree"], dsh, dmeans3D)
            ev = torch.cuda.Event()
            ev.record(side)
        if HOST_TIMES is not None:
            t3 = time.perf_counter()
            for k, v in (("views", t1 - t0), ("collectives", t2 - t1), ("side_stream", t3 - t2)):
                HOST_TIMES[k] = HOST_TIMES.get(k, 0.0) + v
            HOST_TIMES["n"] = HOST_TIMES.get("n", 0) + 1
        # `keep` holds every tensor the side stream touches until wait() has ordered the
        # caller's stream after it (no record_stream per tensor: the handle must be waited,
        # and an unwaited handle waits when it is dropped)
        return (ev, keep, e)


_SIDE = {}


def _side_stream(device):
    if device not in _SIDE:
        _SIDE[device] = torch.cuda.Stream(device=device)
    return _SIDE[device]


class _ShExchangeHandle:
    def __init__(self, parts):
        self.parts = parts

    def wait(self):
        parts, self.parts = self.parts, []
        for ev, _, e in parts:
            if isinstance(ev, _NativeTicket):
                ev.wait()
            elif ev is not None:
                torch.cuda.current_stream().wait_event(ev)
            _check_leaf_grads(e)

    def __del__(self):
        # dropped without wait(): order the current stream after the side stream before the
        # tensors it still uses go back to the caching allocator
        for ev, _, _ in getattr(self, "parts", []):
            if ev is not None:
                try:
                    if isinstance(ev, _NativeTicket):
                        ev.wait()
                    else:
                        torch.cuda.current_stream().wait_event(ev)
                except Exception:
                    pass
        self.parts = []


def _aliases(t, arena):
    """t lies inside the gradient arena's memory (it is one of the backward's views)."""
    a0 = arena.data_ptr()
    return a0 <= t.data_ptr() < a0 + arena.numel() * arena.element_size()


def _check_leaf_grads(e):
    for leaf, before, version in e["watch"]:
        g = leaf.grad
        if g is None or _aliases(g, e["arena"]):
            continue  # untouched (torch.autograd.grad) or handed over without a copy
        if g is before and g._version == version:
            continue  # a .grad from before this backward, not written by it
        raise RuntimeError(
            "ShExchange: autograd copied or accumulated the deferred SH-path gradients into a leaf's .grad "
            "before the exchange completed them (the leaf had a .grad already, or the gradient was reshaped "
            "on its way to the leaf).  Use torch.autograd.grad, zero_grad(set_to_none=True) before "
            "loss.backward(), or gsr_train's arena parameters.")
