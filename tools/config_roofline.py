"""Per-config HBM fractions with the render kernels' bytes counted from the instances they read
(VERDICT r5 Next #5).  SURVEY s8(d) prices the render stages at 52 B x num_rendered, but early
termination (forward.cu:343-359) stops the forward's walk once a tile's pixels are done and the
backward replays only positions below each tile's deepest contributor: at C5 the SURVEY bytes
implied 11.3 TB/s for render_fwd.  Here render_fwd / render_bwd use the instances the kernels
fetch (GSR_STATS build, profiles/round6_fetched_instances.json); every other stage keeps
bench.py's algorithmic_bytes (they do touch every instance or Gaussian).

    python tools/config_roofline.py gpurun_out/configs profiles/round6_fetched_instances.json
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import algorithmic_bytes, HBM_PEAK_GBS  # noqa: E402


def main(cfg_dir, fetched_json):
    fetched = json.load(open(fetched_json))["configs"]
    print(f"# per-stage GB/s and fraction of {HBM_PEAK_GBS:.0f} GB/s; render stages from fetched instances "
          f"({fetched_json}); stage times: the configs run's hipEvent stage pass")
    for cfg in ("c1", "c2", "mt", "c3", "c5"):
        path = os.path.join(cfg_dir, cfg + ".json")
        if not os.path.exists(path) or cfg not in fetched:
            continue
        d = json.load(open(path))
        c, f = d["config"], fetched[cfg]
        P, I, HW, deg = c["P"], c["num_rendered"], c["width"] * c["height"], c["sh_degree"]
        T = ((c["width"] + 15) // 16) * ((c["height"] + 15) // 16)
        W = c.get("written_records")
        tot_b = tot_t = 0.0
        parts = []
        for st, v in d["stages"].items():
            if st == "render_fwd":
                b = algorithmic_bytes(st, P, f["fwd_fetched"], HW, deg)
            elif st == "render_bwd":
                b = algorithmic_bytes(st, P, f["bwd_fetched"], HW, deg)
            else:
                b = algorithmic_bytes(st, P, I, HW, deg, T=T, written=W)
            t = v["avg_ms"] * 1e-3
            tot_b += b
            tot_t += t
            parts.append(f"{st} {b / t / 1e9:.0f} GB/s ({b / t / 1e9 / HBM_PEAK_GBS:.3f})")
        view_b = tot_b
        vps = d["value"]
        print(f"{cfg}: P={P} I={I} fwd_fetched={f['fwd_fetched']} bwd_fetched={f['bwd_fetched']} views/s={vps} "
              f"B_view(fetched)={view_b / 1e9:.3f} GB -> whole view {view_b * vps / 1e9:.0f} GB/s "
              f"({view_b * vps / 1e9 / HBM_PEAK_GBS:.3f})")
        print("   " + "; ".join(parts))


if __name__ == "__main__":
    main(*sys.argv[1:3])
