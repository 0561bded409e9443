"""Re-time every GEGLU entry of miopen_db/kernel_choices.json: K10's fused projection + GEGLU
(``ops.linear_geglu``) against the unfused pair (projection by ``ops.linear`` + the K9 gate), and
rewrite those entries (true = fused).  Run on the MI355X:  python tools/geglu_choose.py OUT.jsonl [--write]"""
import ast
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "video-p2p_amd"))
from vp2p import ops  # noqa: E402

TABLE = os.path.join(ROOT, "miopen_db", "kernel_choices.json")


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
    with open(TABLE) as fh:
        table = json.load(fh)
    torch.set_grad_enabled(False)
    g = torch.Generator(device="cuda").manual_seed(0)
    rows, new = [], {}
    for key in sorted(k for k in table["choices"] if k.startswith("geglu|")):
        _, xs, ws = key.split("|")
        xs, ws = ast.literal_eval(xs), ast.literal_eval(ws)
        x = torch.randn(*xs, device="cuda", generator=g).bfloat16()
        w = (torch.randn(*ws, device="cuda", generator=g) * 0.05).bfloat16()
        b = (torch.randn(ws[0], device="cuda", generator=g) * 0.1).bfloat16()
        wi, bi = ops.geglu_interleave(w, b)
        ok = ops.linear_geglu_supported(x, w)
        t_f = timeit(lambda: ops.linear_geglu(x, wi, bi)) if ok else float("inf")
        t_u = timeit(lambda: ops.geglu(ops.linear(x, w, b)))
        new[key] = bool(t_f < t_u)
        r = dict(key=key, fused_us=round(t_f * 1e3, 2), unfused_us=round(t_u * 1e3, 2), old=table["choices"][key],
                 new=new[key])
        rows.append(r)
        print(json.dumps(r), flush=True)
    with open(out, "w") as fh:
        for r in rows:
            fh.write(json.dumps(r) + "\n")
    if "--write" in sys.argv:
        table["choices"].update(new)
        with open(TABLE, "w") as fh:
            json.dump(table, fh, indent=1)


if __name__ == "__main__":
    main()
