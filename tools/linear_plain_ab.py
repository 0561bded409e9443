"""Plain projections (no residual) at the UNet's shapes: hipBLASLt (F.linear) vs ops.linear's K10 route;
HIP-event medians and max |difference|.  usage: python tools/linear_plain_ab.py OUT.jsonl"""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "video-p2p_amd"))
from vp2p import ops  # noqa: E402


def med(fn, n=20):
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
        ts.append(s.elapsed_time(e) / n * 1e3)
    return sorted(ts)[2]


rows = []
with torch.no_grad():
    shapes = ((131072, 320, 320), (131072, 320, 640), (32768, 640, 640))
    if len(sys.argv) > 2:
        shapes = tuple(tuple(int(v) for v in a.split("x")) for a in sys.argv[2:])
    for M, K, N in shapes:
        x = torch.randn(M, K, device="cuda").bfloat16()
        w = (torch.randn(N, K, device="cuda") * 0.05).bfloat16()
        b = (torch.randn(N, device="cuda") * 0.1).bfloat16()
        t_lib = med(lambda: F.linear(x, w, b))
        t_ops = med(lambda: ops.linear(x, w, b))
        d = (ops.linear(x, w, b).float() - F.linear(x, w, b).float()).abs().max().item()
        r = dict(M=M, K=K, N=N, hipblaslt_us=round(t_lib, 1), ops_linear_us=round(t_ops, 1), maxdiff=d)
        print(json.dumps(r), flush=True)
        rows.append(r)
with open(sys.argv[1], "a") as fh:
    for r in rows:
        fh.write(json.dumps(r) + "\n")
