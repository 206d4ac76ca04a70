"""Per-kernel duration summary of a rocprofv3 --kernel-trace CSV, work launches only.

    python tools/trace_summary.py KERNEL_TRACE_CSV [OUT_TXT]

Launches shorter than 1 % of the kernel's longest launch are the
early exits of the lagged convergence poll (one pass queued past the stop returns
at once); rocprofv3's own --stats averages include them.  This
prints both: all launches and work launches (the bench's HIP events time the
work launches only).
"""
import collections
import csv
import sys


def main():
    path = sys.argv[1]
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        acc[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    lines = [f"{'calls':>6} {'avg_us':>10} {'work':>5} {'work_avg_us':>12} {'work_min':>10} "
             f"{'work_max':>10}  kernel"]
    for k, v in sorted(acc.items(), key=lambda kv: -sum(kv[1])):
        work = [x for x in v if x >= 0.01 * max(v)]
        lines.append(f"{len(v):6d} {sum(v) / len(v):10.1f} {len(work):5d} "
                     f"{sum(work) / len(work):12.1f} {min(work):10.1f} {max(work):10.1f}  {k[:110]}")
    text = "\n".join(lines)
    print(text)
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(text + "\n")


if __name__ == "__main__":
    main()
