"""Per-tile timeline of the depth sort's look-back radix passes (build with -DGSR_SORT_TRACE,
e.g. tools/build_variant.sh strace -DGSR_SORT_TRACE; run with GSR_LIBRARY pointing at it).

Renders the metric scene a few times, then reads, for each pass of the last depth sort and
each tile: entry, tile index taken, ranking done, look-back done, end (s_memrealtime, 100 MHz,
chip-wide).  Prints per pass the span and the phase durations (median / max over tiles), and
the gap between consecutive passes.  usage: python tools/sort_trace.py [config]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "3d_gaussian_magic_change-segment_3dgs_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import harness as Hn  # noqa: E402
from gsr_tools.scene import config_scene_and_camera  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "mt"
    from diff_gaussian_rasterization import _C
    lib = _C._lib
    lib.gsr_sort_trace_read.argtypes = [ctypes.c_void_p, ctypes.c_int]
    scene, cam = config_scene_and_camera(cfg)
    grads = Hn.upstream_grads(cam.height, cam.width)
    buf = np.zeros((5, 1024, 6), np.uint64)
    bbuf = np.zeros((3, 4096, 4), np.uint64)
    lib.gsr_bin_trace_read.argtypes = [ctypes.c_void_p, ctypes.c_int]
    for _ in range(3):
        Hn.run_gsr(scene, cam, grads=grads, want_state=False)
    torch.cuda.synchronize()
    for rep in range(3):
        assert lib.gsr_sort_trace_read(buf.ctypes.data, 1) == 0  # clear
        assert lib.gsr_bin_trace_read(bbuf.ctypes.data, 1) == 0
        Hn.run_gsr(scene, cam, grads=grads, want_state=False)
        torch.cuda.synchronize()
        assert lib.gsr_sort_trace_read(buf.ctypes.data, 0) == 0
        assert lib.gsr_bin_trace_read(bbuf.ctypes.data, 0) == 0
        for k, name in enumerate(("k_rows_scatter", "k_tiles_count", "k_tiles_scatter")):
            m = bbuf[k][:, 0] > 0
            if not m.any():
                continue
            tr = bbuf[k][m].astype(np.int64)
            b0 = tr[:, 0].min()
            s0, s1, e = (tr[:, 0] - b0) / 100, (tr[:, 1] - b0) / 100, (tr[:, 2] - b0) / 100
            nch = tr[:, 3] & 0xFFFF
            dur = e - s0
            print(f"{name}: {m.sum()} blocks, span {e.max():6.2f} us, block entry: median {np.median(s0):6.2f} "
                  f"p90 {np.percentile(s0, 90):6.2f} last {s0.max():6.2f} us; block duration median {np.median(dur):5.2f} "
                  f"max {dur.max():5.2f}; row map {np.median(s1 - s0):5.2f} us; chunks/block mean {nch.mean():.2f} "
                  f"max {nch.max()}; per chunk {np.median((e - s1) / np.maximum(nch, 1)):5.2f} us")
            alive = [int(np.sum((s0 <= t) & (e > t))) for t in np.linspace(0, e.max(), 11)]
            print(f"   blocks alive at 0..100% of span: {alive}")
        used = buf[:, :, 0] > 0
        base = int(buf[:, :, 0][used].min())
        prev_end = None
        print(f"== repetition {rep}")
        for p in (4, 0, 1, 2, 3):
            m = used[p]
            if not m.any():
                continue
            tr = buf[p][m].astype(np.int64)
            rel = lambda c: (tr[:, c] - base) * 10 / 1e3  # us from the first pass's first entry
            s, t1, e = rel(0), rel(1), rel(4)
            copy = tr[:, 2] == 0
            line = (f"{'hist' if p == 4 else f'pass {p}'}: {m.sum()} tiles{' (identity copy)' if copy.all() else ''}, first entry {s.min():7.2f} us, "
                    f"last entry {s.max():7.2f}, last end {e.max():7.2f}, span {e.max() - s.min():6.2f} us")
            if prev_end is not None:
                line += f", gap after previous pass {s.min() - prev_end:5.2f} us"
            print(line)
            prev_end = e.max()
            d_idx = t1 - s
            print(f"   tile index atomic: median {np.median(d_idx):5.2f} max {d_idx.max():5.2f} us")
            if not copy.all():
                r, lb = rel(2), rel(3)
                names = ("load", "LDS hist", "global atomics") if p == 4 else ("load+rank", "look-back", "scatter")
                for name, a, b in zip(names, (t1, r, lb), (r, lb, e)):
                    d = b - a
                    print(f"   {name:10s}: median {np.median(d):5.2f} p90 {np.percentile(d, 90):5.2f} max {d.max():5.2f} us")
                # look-back completion vs tile index: does the chain serialise?
                order = np.argsort(lb)
                print(f"   look-back done at (tile rank 0/25/50/75/100%): "
                      + " ".join(f"{np.percentile(lb, q):6.2f}" for q in (0, 25, 50, 75, 100)))
            else:
                d = e - t1
                print(f"   copy: median {np.median(d):5.2f} max {d.max():5.2f} us")
            print(f"   tiles per XCC: {np.bincount(tr[:, 5] & 15, minlength=8).tolist()}")


if __name__ == "__main__":
    main()
