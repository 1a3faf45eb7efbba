"""Wave timeline of the render kernels (build with -DGSR_WAVE_TRACE, e.g.
tools/build_variant.sh wtrace -DGSR_WAVE_TRACE; run with GSR_LIBRARY pointing at it).

Renders the metric scene (fwd + bwd) a few times, then reads, per wave of the last
launch of k_render_fwd / k_render_bwd: start/end (s_memrealtime, 100 MHz), tile, list
length, deepest list position visited, XCC and HW_ID.  Prints: span, waves alive over
time (how full the chip is), the tail (time with fewer than half the wave slots busy),
duration vs visited depth.  usage: python tools/wave_trace.py [config] [out.npz]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "3d_gaussian_magic_change-segment_3dgs_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import harness as Hn  # noqa: E402
from gsr_tools.scene import config_scene_and_camera  # noqa: E402


def analyse(name, tr, slots):
    t0, t1 = tr[:, 0].astype(np.int64), tr[:, 1].astype(np.int64)
    ok = (t1 > 0) & (t0 > 0)
    tr, t0, t1 = tr[ok], t0[ok], t1[ok]
    base = t0.min()
    s, e = (t0 - base) * 10, (t1 - base) * 10  # ns
    span = e.max()
    dur = e - s
    n = (tr[:, 2] >> 32).astype(np.int64)
    mode = ((tr[:, 2] >> 24) & 255).astype(np.int64)
    depth = (tr[:, 3] & 0xFFFFFF).astype(np.int64)
    xcc = ((tr[:, 3] >> 24) & 15).astype(np.int64)
    hwid = (tr[:, 3] >> 32).astype(np.int64)  # HW_ID: wave[3:0] simd[5:4] cu[11:8] sh[12] se[15:13]
    print(f"== {name}: {len(tr)} waves, span {span / 1e3:.1f} us, wave duration mean {dur.mean() / 1e3:.1f} us, "
          f"max {dur.max() / 1e3:.1f} us, p50 {np.median(dur) / 1e3:.1f}, p90 {np.percentile(dur, 90) / 1e3:.1f}")
    bins = np.arange(0, span + 1000, 1000)
    alive = np.zeros(len(bins))
    for i, b in enumerate(bins):
        alive[i] = np.sum((s <= b) & (e > b))
    print(f"   waves alive (per us): mean {alive.mean():.0f} of {slots} slots; "
          f"time with < {slots // 2} alive: {np.mean(alive < slots // 2) * 100:.0f}% of the span; "
          f"< {slots // 4}: {np.mean(alive < slots // 4) * 100:.0f}%")
    q = np.linspace(0, len(bins) - 1, 11).astype(int)
    print("   alive at 0..100% of span:", " ".join(f"{int(alive[i])}" for i in q))
    last_start = s.max()
    print(f"   last wave starts at {last_start / 1e3:.1f} us ({last_start / span * 100:.0f}% of span); "
          f"start->end of the last 1% of waves: {np.sort(e)[-max(1, len(e) // 100)] / 1e3:.1f}..{span / 1e3:.1f} us")
    # duration model: per visited position
    if depth.max() > 0:
        A = np.vstack([depth, np.ones_like(depth)]).T.astype(np.float64)
        c, *_ = np.linalg.lstsq(A, dur.astype(np.float64), rcond=None)
        print(f"   duration ~ {c[0]:.1f} ns x depth + {c[1] / 1e3:.2f} us; depth mean {depth.mean():.0f} "
              f"max {depth.max()}, list n mean {n.mean():.0f} max {n.max()}")
    print("   waves per XCC:", np.bincount(xcc, minlength=8).tolist())
    for m in sorted(set(mode.tolist())):
        sel = mode == m
        print(f"   mode {m} (quadrants/strips per wave): {sel.sum()} waves, duration mean {dur[sel].mean() / 1e3:.1f} us "
              f"max {dur[sel].max() / 1e3:.1f} us, depth mean {depth[sel].mean():.0f}")
    simd = xcc * 4096 + ((hwid >> 13) & 7) * 512 + ((hwid >> 12) & 1) * 256 + ((hwid >> 8) & 15) * 4 + ((hwid >> 4) & 3)
    ends = {}
    for u, t1 in zip(simd.tolist(), e.tolist()):
        ends[u] = max(ends.get(u, 0), t1)
    work = np.bincount(np.unique(simd, return_inverse=True)[1], weights=dur.astype(np.float64))
    print(f"   SIMDs used {len(ends)}; per-SIMD last end: min {min(ends.values()) / 1e3:.1f} "
          f"median {np.median(list(ends.values())) / 1e3:.1f} max {max(ends.values()) / 1e3:.1f} us; "
          f"per-SIMD sum of wave durations: median {np.median(work) / 1e3:.0f} max {work.max() / 1e3:.0f} us")
    if name == "k_render_bwd":
        # list segments (mode bits 16 front / 32 back): positions replayed = top - seg_lo
        ck = int(os.environ.get("GSR_CKPT", "256"))
        kind = np.where(mode & 32, 2, np.where(mode & 16, 1, 0))
        pos = np.where(kind == 2, np.maximum(depth - ck, 0), depth)
        for kd, lab in ((0, "whole"), (1, "front"), (2, "back")):
            sel = kind == kd
            if sel.any():
                print(f"   {lab:5s}: {sel.sum()} waves, positions mean {pos[sel].mean():.0f} max {pos[sel].max()}, "
                      f"duration mean {dur[sel].mean() / 1e3:.1f} us, start mean {s[sel].mean() / 1e3:.1f} us")
        # the tail: waves still running when the last wave starts
        ls = s.max()
        tail = e > ls
        order = np.argsort(-e[tail])[:12]
        print(f"   {tail.sum()} waves running at the last start ({ls / 1e3:.1f} us); the 12 that end last "
              f"(start us, end us, kind, positions, simd waves alive):")
        for i in order:
            j = np.nonzero(tail)[0][i]
            same = (simd == simd[j]) & (s <= ls) & (e > ls)
            print(f"     {s[j] / 1e3:7.1f} {e[j] / 1e3:7.1f} {('whole', 'front', 'back')[kind[j]]:5s} {pos[j]:4d} "
                  f"{int(same.sum())}")
        # positions still to replay at the last start, per SIMD (linear progress model)
        frac_left = np.clip((e - ls) / np.maximum(e - s, 1), 0, 1) * tail
        left = np.bincount(np.unique(simd, return_inverse=True)[1], weights=frac_left * pos)
        print(f"   positions left at the last start per SIMD: median {np.median(left):.0f} p90 "
              f"{np.percentile(left, 90):.0f} max {left.max():.0f}")
    tile = (tr[:, 2] & 0xFFFFFF).astype(np.int64)
    return dict(start=s, end=e, depth=depth, n=n, xcc=xcc, mode=mode, hwid=hwid, simd=simd, tile=tile)


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "mt"
    out = sys.argv[2] if len(sys.argv) > 2 else None
    from diff_gaussian_rasterization import _C
    lib = _C._lib
    lib.gsr_wave_trace_read.argtypes = [ctypes.c_void_p, ctypes.c_int]
    scene, cam = config_scene_and_camera(cfg)
    grads = Hn.upstream_grads(cam.height, cam.width)
    buf = np.zeros((2, 32768, 4), np.uint64)
    for _ in range(3):
        Hn.run_gsr(scene, cam, grads=grads, want_state=False)
    torch.cuda.synchronize()
    assert lib.gsr_wave_trace_read(buf.ctypes.data, 1) == 0  # clear
    Hn.run_gsr(scene, cam, grads=grads, want_state=False)
    torch.cuda.synchronize()
    assert lib.gsr_wave_trace_read(buf.ctypes.data, 0) == 0
    props = torch.cuda.get_device_properties(0)
    slots = props.multi_processor_count * 4 * 4  # 4 SIMDs per CU x 4 waves per SIMD (the kernels' cap)
    res = {}
    for k, name in enumerate(("k_render_fwd", "k_render_bwd")):
        r = analyse(name, buf[k], props.multi_processor_count * 4 * int(os.environ.get("GSR_BWD_WAVES", "5")) if k == 1 else props.multi_processor_count * 4 * int(os.environ.get("GSR_FWD_WAVES", "5")))
        res.update({f"{name}_{a}": v for a, v in r.items()})
    if out:
        np.savez_compressed(out, **res)


if __name__ == "__main__":
    main()
