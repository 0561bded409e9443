"""K3 (temporal attention + self-replace) at the B4 f8 edit shapes: HIP-event medians and an output
checksum, for an A/B of VP2P_K3_WPB (heads per workgroup).  usage: python tools/k3_wpb_bench.py OUT.jsonl"""
import json
import os
import sys

import torch

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


g = torch.Generator(device="cuda").manual_seed(0)
f, B = 8, 4
with open(sys.argv[1], "a") as fh:
    for C, hw in ((320, 4096), (640, 1024), (1280, 256)):
        qkv = torch.randn(B * f, hw, 3 * C, device="cuda", generator=g).bfloat16()
        q, k, v = qkv[..., :C], qkv[..., C:2 * C], qkv[..., 2 * C:]
        for rep in (False, True):
            fn = lambda: ops.temporal_attention_p2p(q, k, v, f, 8, prompts=2, self_replace=rep)  # noqa: E731
            out = fn()
            t = med(fn)
            r = dict(wpb=os.environ.get("VP2P_K3_WPB", "4"), C=C, hw=hw, self_replace=rep, us=round(t, 2),
                     gbs=round(4 * B * f * hw * C * 2 / t / 1e3, 1), sum=out.double().abs().sum().item())
            fh.write(json.dumps(r) + "\n")
            print(json.dumps(r), flush=True)
