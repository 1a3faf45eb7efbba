"""Split one kernel's dispatches in a rocprofv3 kernel_trace.csv by the bench phase they belong to.

bench.py runs, in order: single-view steps of the metric workload (warm-up, stage pass, timed
steps, then the kernel pass of min(steps, 20) steps whose brackets give the line's avg_launch_ms;
render_bwd then k_gaussian_backward on one stream), the streaming-copy probe, batched steps
(8 render_bwd launches, then k_gaussian_backward_mv, on two overlapping streams) and the training
step legs (a loss gradient, not the metric's upstream gradients). The profiler's kernel_stats average
mixes all of them. This prints, for KERNEL (default k_render_bwd1), each phase's dispatch
durations, the metric phase's last N launches (N = --kpass, default 20) = the kernel pass, and the N
before them = the timed region (bench.py --steps N).

usage: python tools/ktrace_phases.py kernel_trace.csv [KERNEL] [--kpass N]
"""
import csv
import statistics
import sys


def stats(v):
    return (f"dispatches={len(v):4d} mean_us={statistics.fmean(v):8.2f} "
            f"median_us={statistics.median(v):8.2f} min={min(v):8.2f} max={max(v):8.2f}")


def main():
    args = [a for a in sys.argv[1:]]
    kpass = 20
    if "--kpass" in args:
        i = args.index("--kpass")
        kpass = int(args[i + 1])
        del args[i:i + 2]
    path = args[0]
    kern = args[1] if len(args) > 1 else "k_render_bwd1"
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Dispatch_Id"]))
    phases, pending = [], []   # phases: [kind, [durations]] in dispatch order

    def add(kind, v):
        if not v:
            return
        if phases and phases[-1][0] == kind:
            phases[-1][1].extend(v)
        else:
            phases.append([kind, list(v)])

    for r in rows:
        name = r["Kernel_Name"]
        if kern in name:
            pending.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        elif "k_gaussian_backward_mv" in name:
            add("batched", pending)
            pending = []
        elif "k_gaussian_backward" in name:
            add("single", pending)
            pending = []
        elif "k_stream_copy" in name or "k_adam" in name:
            phases.append(["other", []])
    phases = [p for p in phases if p[1]]
    groups = {}
    for i, (kind, v) in enumerate(phases):
        label = "metric" if (i == 0 and kind == "single") else (
            "train-step legs" if kind == "single" else kind)
        groups.setdefault(label, []).extend(v)
    for label, v in groups.items():
        print(f"{kern} {label:16s} {stats(v)}")
    if phases and phases[0][0] == "single" and len(phases[0][1]) >= kpass:
        print(f"{kern} metric kernel pass (last {kpass}) {stats(phases[0][1][-kpass:])}")
        if len(phases[0][1]) >= 2 * kpass:  # the timed region's steps precede the kernel pass
            print(f"{kern} metric timed region (the {kpass} before) {stats(phases[0][1][-2 * kpass:-kpass])}")
    if pending:
        print(f"{kern} unclassified dispatches={len(pending)}")


if __name__ == "__main__":
    main()
