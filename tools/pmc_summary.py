"""Summarise rocprofv3 counter CSVs (tools/pmc.sh) per gsr kernel -> JSON.

HBM bytes per launch = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024: on gfx950 FETCH_SIZE
reports half the bytes of wide coalesced reads (MI355X_MICROARCH.md, HBM section);
other access widths are uncalibrated, so the raw numbers are kept beside it."""
import csv, glob, json, os, sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PMC = os.environ.get("GSR_PMC_DIR", os.path.join(ROOT, "gpurun_out", "pmc"))  # (tools/pmc_cfg.sh: gpurun_out/pmc_CONFIG)
STAGE_OF = {"k_render_bwd": "render_bwd", "k_render_bwd1": "render_bwd", "k_render_fwd": "render_fwd", "k_gaussian_backward": "gaussian_bwd",
            "k_preprocess": "preprocess", "k_duplicate": "duplicate", "k_tile_order": "ranges", "k_tile_order_counted": "ranges", "k_scan": "scan", "k_radix_hist": "radix_hist",
            "k_radix_scatter": "radix_scatter", "k_radix_upsweep": "radix_upsweep", "k_adam": "adam_step",
            "k_activation_backward": "activation_backward"}


def short(name):
    n = name.replace("gsr::(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0].split("<")[0]


def load(sub):
    files = glob.glob(os.path.join(PMC, sub, "**", "*counter_collection.csv"), recursive=True)
    acc = defaultdict(lambda: defaultdict(list))
    for f in files:
        for r in csv.DictReader(open(f)):
            k = short(r.get("Kernel_Name", r.get("Kernel-Name", "")))
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return acc


def sources_sha256():
    """Hash of the HIP sources the counters were collected on (bench.py compares it with
    the build it times before reporting the counter-derived fields)."""
    import hashlib
    h = hashlib.sha256()
    csrc = os.path.join(ROOT, "3d_gaussian_magic_change-segment_3dgs_amd", "csrc")
    for f in sorted(os.listdir(csrc)):
        if f.endswith((".hip", ".h")) and not f.startswith("."):
            h.update(f.encode())
            h.update(open(os.path.join(csrc, f), "rb").read())
    h.update(open(os.path.join(ROOT, "include", "gsr.h"), "rb").read())
    return h.hexdigest()


def main():
    out = {"note": __doc__.strip(), "sources_sha256": sources_sha256(), "kernels": {}}
    merged = defaultdict(dict)
    for sub in ("fetch", "write", "sq"):
        for k, cs in load(sub).items():
            for c, vals in cs.items():
                # counters are reported per dispatch (possibly per XCD/SE dimension): sum per dispatch
                merged[k][c] = sum(vals) / max(1, len(vals)) if c.startswith("SQ_") else sum(vals) / max(1, len(vals))
    # per-dispatch means: re-aggregate by dispatch count from the kernel traces
    for k, cs in merged.items():
        stage = STAGE_OF.get(k, k)
        d = {c: v for c, v in cs.items()}
        if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
            d["hbm_bytes_per_launch"] = 2 * d["FETCH_SIZE"] * 1024 + d["WRITE_SIZE"] * 1024
            d["hbm_bytes_per_launch_raw"] = (d["FETCH_SIZE"] + d["WRITE_SIZE"]) * 1024
        out["kernels"][stage] = d
    json.dump(out, open(sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "profiles", "round1_pmc_summary.json"), "w"), indent=1)
    for k, d in out["kernels"].items():
        print(k, {c: (round(v / 1e6, 3) if "bytes" in c else round(v, 1)) for c, v in d.items()})


if __name__ == "__main__":
    main()
