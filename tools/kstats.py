"""Summarise a rocprofv3 kernel_stats.csv: one line per gsr kernel (short name, calls, avg/min/max us).
--per-step K: also each kernel's time per call of kernel K (one call per step) and their sum."""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    n = r["Name"]
    if "at::" in n and "--all" not in sys.argv:
        continue
    m = re.search(r"(k_[A-Za-z0-9_]+)(<[^>]*>)?", n)
    short = (m.group(1) + (m.group(2) or "")) if m else n[:50]
    print(f"{short:44s} calls={r['Calls']:>5s} avg_us={float(r['AverageNs']) / 1e3:8.2f} "
          f"min={float(r['MinNs']) / 1e3:8.2f} max={float(r['MaxNs']) / 1e3:8.2f}")

if "--per-step" in sys.argv:
    k = sys.argv[sys.argv.index("--per-step") + 1]
    steps = sum(int(r["Calls"]) for r in rows if k in r["Name"])
    tot = 0.0
    for r in rows:
        if "at::" in r["Name"] or "stream_copy" in r["Name"] or "rocclr" in r["Name"]:
            continue
        t = float(r["TotalDurationNs"]) / 1e3 / max(steps, 1)
        tot += t
    print(f"sum of gsr kernels per {k} call: {tot:.1f} us over {steps} steps")
