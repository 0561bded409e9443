"""Per-shape K7/K8 kernel durations from a rocprofv3 --kernel-trace database of tools/norm_shapes.py
(A/B mode: the other build's launches precede the in-tree library's for every shape).
usage: python tools/norm_shapes_report.py DB SHAPES_TXT N AB(0|1)"""
import json
import sqlite3
import sys


def main(db, shapes_txt, n, ab):
    cur = sqlite3.connect(db).cursor()
    ks = [(r[0], (r[2] - r[1]) / 1e3) for r in cur.execute("select name, start, end from kernels order by start")
          if "gn_" in r[0] or "ln_kernel" in r[0]]
    shapes = [json.loads(line) for line in open(shapes_txt) if line.startswith("{")]
    variants = ("A", "B") if ab else ("B",)
    i = 0
    med = lambda v: sorted(v)[len(v) // 2]  # noqa: E731
    for s in shapes:
        xb = s["x_bytes"]
        for var in variants:
            if s["op"] == "gn":
                for mode in ("add+silu", "plain"):
                    st = [ks[i + 2 * j][1] for j in range(n)]
                    ap = [ks[i + 2 * j + 1][1] for j in range(n)]
                    i += 2 * n
                    print(json.dumps({"op": "gn " + mode, "lib": var, "C": s["C"], "H": s["H"], "MB": round(xb / 1e6, 1),
                                      "stats_us": round(med(st), 1), "stats_GBps": round(xb / med(st) / 1e3),
                                      "apply_us": round(med(ap), 1), "apply_GBps": round(2 * xb / med(ap) / 1e3)}))
            else:
                t = med([k[1] for k in ks[i:i + n]])
                i += n
                print(json.dumps({"op": "ln", "lib": var, "C": s["C"], "H": s["H"], "us": round(t, 1),
                                  "GBps": round(2 * xb / t / 1e3)}))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]))
