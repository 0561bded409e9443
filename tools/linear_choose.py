"""Time every plain projection shape of the UNet3D on K10's GEMM core (``ops.linear_k10``, the tile
K10 picks itself) against hipBLASLt (``F.linear``) over a range of row counts M, and write the
``linear_rules`` of ``miopen_db/kernel_choices.json`` that ``vp2p.ops.LinearRule`` reads: per (K, N),
the runs of consecutive measured M over which K10 is faster by > 2 % (open-ended at the measured
extremes).  ``--from OLD.jsonl`` recomputes the rules from a committed measurement; with ``--ms M1,M2,..``
as well, only those row counts are measured and merged into OLD's rows (the other M keep OLD's
timings, so decisions at OLD's measured M do not move).

Run on the MI355X:  python tools/linear_choose.py OUT.jsonl [--write] [--from OLD.jsonl --ms 768,3072]"""
import json
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "video-p2p_amd"))
from vp2p import ops  # noqa: E402

# (K, N) of every nn.Linear on the UNet path: per resolution C = 320 / 640 / 1280:
#   to_q / to_out / proj_in / proj_out (C, C), frame-0 K|V (C, 2C), attn_temp qkv (C, 3C),
#   FF out (4C, C), GEGLU projection (C, 8C); the cross-attention context K|V (768, 2C)
PAIRS = []
for C in (320, 640, 1280):
    PAIRS += [(C, C), (C, 2 * C), (C, 3 * C), (4 * C, C), (C, 8 * C)]
MS = (2048, 4096, 8192, 16384, 32768, 65536, 131072, 262144)


def timeit(fn, n=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(n):
            fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e) / n)
    return sorted(ts)[2]


def main():
    out = sys.argv[1]
    write = "--write" in sys.argv
    rows = []
    ms = None
    if "--ms" in sys.argv:
        ms = tuple(int(m) for m in sys.argv[sys.argv.index("--ms") + 1].split(","))
    if "--from" in sys.argv:
        with open(sys.argv[sys.argv.index("--from") + 1]) as fh:
            rows = [json.loads(line) for line in fh]
    if ms is not None or not rows:
        new = measure(ms or MS)
        keys = {(r["M"], r["K"], r["N"]) for r in new}
        rows = [r for r in rows if (r["M"], r["K"], r["N"]) not in keys] + new
        with open(out, "w") as fh:
            for r in rows:
                fh.write(json.dumps(r) + "\n")
    write_rules(rows, write)


def measure(ms):
    g = torch.Generator(device="cuda").manual_seed(0)
    rows = []
    torch.set_grad_enabled(False)
    for K, N in PAIRS:
        w = (torch.randn(N, K, device="cuda", generator=g) * 0.05).bfloat16()
        b = (torch.randn(N, device="cuda", generator=g) * 0.1).bfloat16()
        for M in ms:
            if M * max(K, N) * 2 > 2 ** 31:
                continue
            x = torch.randn(M, K, device="cuda", generator=g).bfloat16()
            t_k = timeit(lambda: ops.linear_k10(x, w, b))
            t_l = timeit(lambda: F.linear(x, w, b))
            d = (ops.linear_k10(x, w, b).float() - F.linear(x, w, b).float()).abs().max().item()
            r = dict(M=M, K=K, N=N, k10_us=round(t_k * 1e3, 2), hipblaslt_us=round(t_l * 1e3, 2),
                     k10_tflops=round(2.0 * M * K * N / t_k / 1e9, 1), maxdiff=d)
            rows.append(r)
            print(json.dumps(r), flush=True)
            del x
    return rows


def write_rules(rows, write):
    rules = {}
    for K, N in PAIRS:
        rs = sorted((r for r in rows if r["K"] == K and r["N"] == N), key=lambda r: r["M"])
        runs, cur = [], None
        for i, r in enumerate(rs):
            win = r["k10_us"] < 0.98 * r["hipblaslt_us"]
            if win and cur is None:
                cur = [None if i == 0 else r["M"], r["M"]]
            elif win:
                cur[1] = r["M"]
            if (not win or i == len(rs) - 1) and cur is not None:
                if win and i == len(rs) - 1:
                    cur[1] = None
                runs.append(cur)
                cur = None
        if runs:
            rules[f"{K}|{N}"] = runs
    print("linear_rules", json.dumps(rules))
    if write:
        path = os.path.join(ROOT, "miopen_db", "kernel_choices.json")
        with open(path) as fh:
            table = json.load(fh)
        table["linear_rules"] = rules
        table["linear_how"] = ("tools/linear_choose.py on an MI355X: per (K, N), the ranges of M over which "
                               "K10 (its own tile choice) beat hipBLASLt by > 2 % at every measured M")
        with open(path, "w") as fh:
            json.dump(table, fh, indent=1)


if __name__ == "__main__":
    main()
