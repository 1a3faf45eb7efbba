"""How far integer outputs move under the reference binary's FMA contraction (VERDICT r5 Next #1).

DGR is compiled by nvcc with its defaults (DGR/setup.py:17-34: --fmad=true), so the reference
binary evaluates the projection (auxiliary.h:58-77), computeCov3D / computeCov2D
(forward.cu:74-152), the determinant / eigenvalue / radius lines (forward.cu:219-232) and the
blend's power (forward.cu:346) with fused multiply-adds.  gsr and its oracle round every
product separately.  `radius = ceil(3 sqrt(lambda))` and getRect's (int) truncation
(auxiliary.h:46-56) flip on last-bit changes, and the depth bits are the low half of the sort
key (rasterizer_impl.cu:98-108), so this module measures, between two runs of the same view:

* Gaussians whose visibility, radius, tile rectangle or tiles_touched differ ("moved");
* Gaussians whose depth bits differ (key low bits; they reorder a tile only when two depths
  are within a few ulps);
* the change of num_rendered;
* tiles whose point_list differs, each EXPLAINED either by a moved Gaussian whose old or new
  rectangle covers the tile, or by an order swap of two Gaussians whose depths are within
  SWAP_ULPS ulps (same set of Gaussians); any other difference is "unexplained";
* pixels whose n_contrib differs, and how many of them lie outside the differing tiles.

TEST INFRASTRUCTURE (imported by tests/ and tools/contract_report.py only).
"""
import numpy as np

SWAP_ULPS = 8


def rects(px, py, radii, W, H):
    """getRect (auxiliary.h:46-56) in float32 with (int) truncation and the grid clamp."""
    gx, gy = (W + 15) // 16, (H + 15) // 16
    rad = radii.astype(np.float32)
    f16 = np.float32(16)
    px, py = px.astype(np.float32), py.astype(np.float32)
    clip = lambda v, n: np.clip(np.trunc(v).astype(np.int64), 0, n)
    x0, x1 = clip((px - rad) / f16, gx), clip((px + rad + np.float32(15)) / f16, gx)
    y0, y1 = clip((py - rad) / f16, gy), clip((py + rad + np.float32(15)) / f16, gy)
    vis = radii > 0
    z = np.zeros_like(x0)
    return (np.where(vis, x0, z), np.where(vis, y0, z), np.where(vis, x1, z), np.where(vis, y1, z))


def from_oracle(run, W, H):
    m2 = run.get("means2D").reshape(-1, 2)
    return {"radii": run.radii.astype(np.int64), "px": m2[:, 0], "py": m2[:, 1],
            "depth": run.get("depths").astype(np.float32), "tiles_touched": run.get("tiles_touched").astype(np.int64),
            "point_list": run.get("point_list").astype(np.int64), "ranges": run.get("ranges").reshape(-1, 2).astype(np.int64),
            "n_contrib": run.get("n_contrib").reshape(H, W).astype(np.int64), "num_rendered": int(run.num_rendered)}


def from_gsr(g):
    rec = g["rec"].reshape(-1, 16)
    vis = g["radii"] > 0
    return {"radii": g["radii"].astype(np.int64), "px": rec[:, 0], "py": rec[:, 1],
            "depth": np.where(vis, rec[:, 6], np.float32(0)).astype(np.float32),
            "tiles_touched": g["tiles_touched"].astype(np.int64),
            "point_list": g["point_list"].astype(np.int64), "ranges": g["ranges"].reshape(-1, 2).astype(np.int64),
            "n_contrib": g["n_contrib"].astype(np.int64), "num_rendered": int(g["num_rendered"])}


def _ulps(a, b):
    """|a - b| in float32 ulps of the larger magnitude (positive depths)."""
    a, b = np.float32(a), np.float32(b)
    return abs(int(a.view(np.int32)) - int(b.view(np.int32)))


def compare(base, other, W, H):
    """Statistics of `other` against `base` (dicts from from_oracle / from_gsr)."""
    gx, gy = (W + 15) // 16, (H + 15) // 16
    ra = rects(base["px"], base["py"], base["radii"], W, H)
    rb = rects(other["px"], other["py"], other["radii"], W, H)
    vis_a, vis_b = base["radii"] > 0, other["radii"] > 0
    rect_diff = np.zeros(vis_a.shape, bool)
    for u, v in zip(ra, rb):
        rect_diff |= u != v
    moved = (vis_a != vis_b) | (base["radii"] != other["radii"]) | rect_diff | \
        (base["tiles_touched"] != other["tiles_touched"])
    both = vis_a & vis_b
    depth_diff = both & (base["depth"].view(np.uint32) != other["depth"].view(np.uint32))
    st = {"P": int(vis_a.size), "visible": int(vis_a.sum()), "moved": int(moved.sum()),
          "visibility_changed": int((vis_a != vis_b).sum()), "radius_changed": int((base["radii"] != other["radii"]).sum()),
          "rect_changed": int(rect_diff.sum()), "tiles_touched_changed": int((base["tiles_touched"] != other["tiles_touched"]).sum()),
          "depth_bits_changed": int(depth_diff.sum()), "num_rendered": base["num_rendered"],
          "d_num_rendered": other["num_rendered"] - base["num_rendered"]}
    # tiles covered by a moved Gaussian's old or new rectangle
    touched = np.zeros((gy + 1, gx + 1), np.int64)
    for (x0, y0, x1, y1) in (ra, rb):
        idx = np.nonzero(moved & (x1 > x0) & (y1 > y0))[0]
        np.add.at(touched, (y0[idx], x0[idx]), 1)
        np.add.at(touched, (y0[idx], x1[idx]), -1)
        np.add.at(touched, (y1[idx], x0[idx]), -1)
        np.add.at(touched, (y1[idx], x1[idx]), 1)
    touched = (touched.cumsum(0).cumsum(1)[:gy, :gx] > 0).reshape(-1)
    T = gx * gy
    pa, pb = base["point_list"], other["point_list"]
    rga, rgb = base["ranges"], other["ranges"]
    len_a, len_b = rga[:, 1] - rga[:, 0], rgb[:, 1] - rgb[:, 0]
    diff_tiles, by_moved, by_swap, unexplained, max_swap_ulps = [], 0, 0, [], 0
    # fast path: tiles whose lists are equal need no work
    cand = np.nonzero(len_a != len_b)[0].tolist()
    same_len = np.nonzero((len_a == len_b) & (len_a > 0))[0]
    if same_len.size:  # equal-length tiles compared instance-wise at once, reduced per tile
        tile_of = np.repeat(same_len, len_a[same_len])
        off = np.arange(tile_of.size) - np.repeat(np.cumsum(len_a[same_len]) - len_a[same_len], len_a[same_len])
        bad = np.unique(tile_of[pa[rga[tile_of, 0] + off] != pb[rgb[tile_of, 0] + off]])
        cand += bad.tolist()
    da = base["depth"]
    for t in sorted(set(cand)):
        la, lb = pa[rga[t, 0]:rga[t, 1]], pb[rgb[t, 0]:rgb[t, 1]]
        if np.array_equal(la, lb):
            continue
        diff_tiles.append(t)
        if touched[t]:
            by_moved += 1
            continue
        ok = la.size == lb.size and np.array_equal(np.sort(la), np.sort(lb))
        if ok:  # same set: every inverted pair must be a near-tie in depth
            w = np.nonzero(la != lb)[0]
            lo, hi = int(w[0]), int(w[-1]) + 1
            rank_b = {int(g): i for i, g in enumerate(lb[lo:hi])}
            win = [int(g) for g in la[lo:hi]]
            for i in range(len(win)):
                for j in range(i + 1, len(win)):
                    if rank_b[win[i]] > rank_b[win[j]]:
                        u = _ulps(da[win[i]], da[win[j]])
                        max_swap_ulps = max(max_swap_ulps, u)
                        if u > SWAP_ULPS:
                            ok = False
        if ok:
            by_swap += 1
        else:
            unexplained.append(t)
    nca, ncb = base["n_contrib"], other["n_contrib"]
    pix_diff = nca != ncb
    tile_mask = np.zeros(T, bool)
    tile_mask[diff_tiles] = True
    tile_img = np.repeat(np.repeat(tile_mask.reshape(gy, gx), 16, 0), 16, 1)[:H, :W]
    st.update({"tiles": T, "tiles_diff": len(diff_tiles), "tiles_by_moved": by_moved, "tiles_by_swap": by_swap,
               "tiles_unexplained": len(unexplained), "max_swap_ulps": max_swap_ulps,
               "pixels": int(H * W), "n_contrib_diff": int(pix_diff.sum()),
               "n_contrib_diff_outside_diff_tiles": int((pix_diff & ~tile_img).sum())})
    st["_moved"] = moved
    st["_unexplained"] = unexplained
    return st


def summary(st):
    return {k: v for k, v in st.items() if not k.startswith("_")}
