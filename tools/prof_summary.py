"""Summarise a rocprofv3 --kernel-trace database (or kernel_stats.csv) into a per-kernel table."""
import csv
import glob
import os
import sqlite3
import sys


def from_db(path):
    cur = sqlite3.connect(path).cursor()
    return [(r[0], r[1], r[2], r[3]) for r in cur.execute(
        "select name, count(*), sum(end-start), avg(end-start) from kernels group by name")]


def from_csv(path):
    rows = []
    for r in csv.DictReader(open(path)):
        rows.append((r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]), float(r["AverageNs"])))
    return rows


def main(src, out=None, top=40):
    rows = from_db(src) if src.endswith(".db") else from_csv(src)
    rows.sort(key=lambda r: -r[2])
    tot = sum(r[2] for r in rows)
    lines = [f"# source: {os.path.basename(src)}  total kernel time {tot / 1e6:.1f} ms  kernels {len(rows)}",
             f"{'total_ms':>10} {'pct':>6} {'calls':>7} {'avg_us':>10}  name"]
    for name, n, t, avg in rows[:top]:
        lines.append(f"{t / 1e6:10.2f} {100 * t / tot:6.2f} {n:7d} {avg / 1e3:10.2f}  {name[:150]}")
    text = "\n".join(lines) + "\n"
    if out:
        open(out, "w").write(text)
    print(text)


if __name__ == "__main__":
    src = sys.argv[1]
    if os.path.isdir(src):
        cand = glob.glob(os.path.join(src, "**", "*kernel_stats.csv"), recursive=True) or \
            glob.glob(os.path.join(src, "**", "*.db"), recursive=True)
        src = cand[0]
    main(src, sys.argv[2] if len(sys.argv) > 2 else None)
