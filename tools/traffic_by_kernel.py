"""HBM-side traffic of every kernel of a run, by launch shape, from two rocprofv3 --pmc passes.

usage: python tools/traffic_by_kernel.py FETCH_CSV WRITE_CSV [TOP]
Groups dispatches by (kernel name, grid size); per group: calls, mean duration (from the FETCH pass),
FETCH_SIZE x 2 (the gfx950 correction for wide coalesced reads, MI355X_MICROARCH.md HBM section;
it over-counts scattered 16-B reads) and WRITE_SIZE per launch in MB, and the rate they imply.
Sorted by total time, so the kernels whose traffic matters come first.
"""
import csv
import sys


def short(name):
    n = name.replace("void ", "")
    cut = n.find("(")
    return (n[:cut] if cut > 0 else n)[:64]


def load(path, counter):
    per = {}
    with open(path) as fh:
        for row in csv.DictReader(fh):
            if row["Counter_Name"] != counter:
                continue
            d = row["Dispatch_Id"]
            e = per.setdefault(d, {"key": (short(row["Kernel_Name"]), int(row["Grid_Size"])), "v": 0.0,
                                   "t": (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-9})
            e["v"] += float(row["Counter_Value"])
    return per


def main():
    fe, wr = load(sys.argv[1], "FETCH_SIZE"), load(sys.argv[2], "WRITE_SIZE")
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    groups = {}
    for d in fe.values():
        g = groups.setdefault(d["key"], {"n": 0, "t": 0.0, "f": 0.0, "w": 0.0, "nw": 0})
        g["n"] += 1
        g["t"] += d["t"]
        g["f"] += 2 * 1024 * d["v"]
    for d in wr.values():
        g = groups.get(d["key"])
        if g is not None:
            g["w"] += 1024 * d["v"]
            g["nw"] += 1
    tot = sum(g["t"] for g in groups.values())
    print(f"{'kernel':64s} {'grid':>9s} {'calls':>6s} {'us':>8s} {'share':>6s} {'fetchMB':>9s} {'writeMB':>8s} {'TB/s':>6s}")
    for k, g in sorted(groups.items(), key=lambda kv: -kv[1]["t"])[:top]:
        t = g["t"] / g["n"]
        f = g["f"] / g["n"] / 1e6
        w = g["w"] / max(g["nw"], 1) / 1e6
        print(f"{k[0]:64s} {k[1]:9d} {g['n']:6d} {t * 1e6:8.1f} {g['t'] / tot:6.3f} {f:9.1f} {w:8.1f} {(f + w) / 1e6 / t:6.2f}")


if __name__ == "__main__":
    main()
