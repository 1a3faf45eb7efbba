"""Gap analysis of a rocprofv3 kernel trace (kt_kernel_trace.csv): per step, GPU
busy time vs wall time between the first and last kernel, and the largest idle gaps
between consecutive kernels (by kernel pair)."""
import csv, glob, sys
from collections import defaultdict

path = sys.argv[1] if len(sys.argv) > 1 else glob.glob("gpurun_out/prof/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(path)))
ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
              r["Kernel_Name"].replace("gsr::(anonymous namespace)::", "").split("(")[0][:40]) for r in rows))
# steps start at k_preprocess
starts = [i for i, k in enumerate(ks) if k[2].startswith("k_preprocess")]
steps = [(starts[i], starts[i + 1]) for i in range(len(starts) - 1)][-10:]
gap = defaultdict(list)
tot_wall = tot_busy = 0
for a, b in steps:
    seg = ks[a:b]
    wall = seg[-1][1] - seg[0][0]
    busy = sum(e - s for s, e, _ in seg)
    tot_wall += wall
    tot_busy += busy
    for (s0, e0, n0), (s1, e1, n1) in zip(seg, seg[1:]):
        gap[(n0, n1)].append(s1 - e0)
    # gap to next step's first kernel
print(f"steps={len(steps)} mean wall (first->last kernel) {tot_wall / len(steps) / 1e3:.1f} us, "
      f"busy {tot_busy / len(steps) / 1e3:.1f} us, kernels/step {steps[0][1] - steps[0][0]}")
if len(starts) > 1:
    cyc = [ks[starts[i + 1]][0] - ks[starts[i]][0] for i in range(len(starts) - 1)][-10:]
    print(f"step period (preprocess->preprocess) {sum(cyc) / len(cyc) / 1e3:.1f} us")
items = sorted(gap.items(), key=lambda kv: -sum(kv[1]) / len(kv[1]))
for (n0, n1), v in items[:25]:
    print(f"  {sum(v) / len(v) / 1e3:8.1f} us  {n0} -> {n1}")

# per-kernel durations in the last step (launch order)
a, b = steps[-1]
print("last step kernels:")
for s0, e0, n0 in ks[a:b]:
    print(f"  {(e0 - s0) / 1e3:8.1f} us  {n0}")
