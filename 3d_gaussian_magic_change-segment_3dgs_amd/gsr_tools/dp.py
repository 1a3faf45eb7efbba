"""View-parallel data parallelism for the rasterizer.

Each rank renders its own view of the replicated Gaussians; the only exchange is
one all-reduce (sum) of the parameter-gradient bucket
[dmeans3D | dsh | dopacity | dscales | drot | dsegments] (61 f32 / Gaussian at SH3).
The backward writes every gradient into one arena whose first `bucket` floats are
exactly that bucket (diff_gaussian_rasterization._C.grad_arena_layout), so the
all-reduce runs in place with no packing copy.  Backend "nccl" is RCCL over xGMI on
ROCm; "gloo" is used for the CPU tests.
"""
import torch
import torch.distributed as dist


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
        dist.all_reduce(g, op=dist.ReduceOp.SUM, group=group)
    return g


def reduce_densification_stats(xyz_gradient_accum, denom, max_radii2D, group=None):
    """Combine per-rank densification statistics before densify_and_prune
    (SURVEY.md s8e): accumulated view-space gradient norms and view counts are
    summed, max_radii2D is max-reduced.  Each rank accumulated its own views'
    |dmeans2D| before any reduction, as the reference does per view."""
    both = torch.cat([xyz_gradient_accum.reshape(-1), denom.reshape(-1)])
    dist.all_reduce(both, op=dist.ReduceOp.SUM, group=group)
    n = xyz_gradient_accum.numel()
    xyz_gradient_accum.copy_(both[:n].view_as(xyz_gradient_accum))
    denom.copy_(both[n:].view_as(denom))
    dist.all_reduce(max_radii2D, op=dist.ReduceOp.MAX, group=group)
