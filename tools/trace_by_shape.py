"""Per-launch-shape summary of rocprofv3 kernel traces, side by side: for each (kernel, grid) the
launch count, the mean duration and the mean time per workgroup, so two runs of different sizes
(e.g. the 8- and 24-frame edits) compare per unit of work.
usage: python tools/trace_by_shape.py A/run_kernel_trace.csv [B/run_kernel_trace.csv ...]"""
import collections
import csv
import re
import sys


def short(name):
    name = re.sub(r"\(.*", "", name)
    name = re.sub(r"^void ", "", name)
    return name[:60]


def load(path):
    agg = collections.defaultdict(list)
    for row in csv.DictReader(open(path)):
        wg = 1
        for ax in "XYZ":
            g, w = int(row[f"Grid_Size_{ax}"]), max(1, int(row[f"Workgroup_Size_{ax}"]))
            wg *= (g + w - 1) // w
        dur = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-3
        agg[(short(row["Kernel_Name"]), wg)].append(dur)
    return agg


def main():
    runs = [load(p) for p in sys.argv[1:]]
    totals = [collections.defaultdict(float) for _ in runs]
    for t, agg in zip(totals, runs):
        for (k, _), d in agg.items():
            t[k] += sum(d)
    kernels = sorted({k for t in totals for k in t}, key=lambda k: -max(t.get(k, 0.0) for t in totals))
    print("kernel totals (ms):", " | ".join(sys.argv[1:]))
    for k in kernels[:30]:
        print(f"  {k:60s} " + " ".join(f"{t.get(k, 0.0) / 1e3:9.2f}" for t in totals))
    print("\nper launch shape: kernel, workgroups -> calls, mean us, us per 1000 workgroups (per run)")
    for k in kernels[:14]:
        shapes = sorted({wg for agg in runs for (kk, wg) in agg if kk == k})
        for wg in shapes:
            cells = []
            for agg in runs:
                d = agg.get((k, wg))
                cells.append("-" if not d else f"{len(d):5d} {sum(d) / len(d):9.1f} {sum(d) / len(d) / wg * 1e3:8.2f}")
            print(f"  {k[:48]:48s} {wg:7d}  " + "  |  ".join(cells))


if __name__ == "__main__":
    main()
