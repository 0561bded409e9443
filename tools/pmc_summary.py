"""Mean per-dispatch PMC counters of one kernel from rocprofv3 --pmc csv directories.

usage: python tools/pmc_summary.py KERNEL_SUBSTR DIR [DIR...]
Also prints the effective clock (GRBM_GUI_ACTIVE / 8 XCDs / kernel duration) when both are present.
"""
import csv
import glob
import os
import sys


def load(d, sub):
    vals, n = {}, {}
    for row in csv.DictReader(open(glob.glob(os.path.join(d, "*counter_collection.csv"))[0])):
        if sub not in row["Kernel_Name"]:
            continue
        c = row["Counter_Name"]
        key = (c, row["Dispatch_Id"])
        vals[key] = vals.get(key, 0.0) + float(row["Counter_Value"])
    out = {}
    for (c, _), v in vals.items():
        out.setdefault(c, []).append(v)
    durs = []
    kt = glob.glob(os.path.join(d, "*kernel_trace.csv"))
    if kt:
        for row in csv.DictReader(open(kt[0])):
            if sub in row["Kernel_Name"]:
                durs.append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-9)
    return {c: sum(v) / len(v) for c, v in out.items()}, durs


def main():
    sub = sys.argv[1]
    for d in sys.argv[2:]:
        m, durs = load(d, sub)
        print(f"# {d}")
        for c in sorted(m):
            print(f"  {c:28s} {m[c]:18.1f}")
        if durs:
            t = sum(durs) / len(durs)
            print(f"  {'duration_ms':28s} {t * 1e3:18.4f}")
            if "GRBM_GUI_ACTIVE" in m:
                print(f"  {'effective_clock_GHz':28s} {m['GRBM_GUI_ACTIVE'] / 8 / t / 1e9:18.3f}")


if __name__ == "__main__":
    main()
