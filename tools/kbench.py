"""Kernel microbenchmarks at the edit workload's shapes (B=4 prompts x CFG, f frames, 512^2)."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "video-p2p_amd"))
from vp2p import ops, _lib  # noqa: E402


def timeit(fn, iters=20, warmup=3):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e-3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=8)
    ap.add_argument("--dtype", default="bf16")
    args = ap.parse_args()
    dt = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    B, f, heads = 4, args.frames, 8
    res = []
    for hw, C in ((4096, 320), (1024, 640), (256, 1280), (64, 1280)):
        d = C // heads
        q = torch.randn(B * f, hw, C, device="cuda", dtype=dt)
        k0 = torch.randn(B, hw, C, device="cuda", dtype=dt)
        v0 = torch.randn(B, hw, C, device="cuda", dtype=dt)
        qs = (q.float() * ops.frame_query_scale(d)).to(dt)
        t = timeit(lambda: ops.frame_attention(qs, k0, v0, f, heads, q_prescaled=True))
        fl = 4.0 * B * f * hw * hw * C
        res.append(dict(kernel="frame_attn", hw=hw, d=d, ms=t * 1e3, tflops=fl / t / 1e12))
        kc = torch.randn(B, 77, C, device="cuda", dtype=dt)
        vc = torch.randn(B, 77, C, device="cuda", dtype=dt)
        t = timeit(lambda: ops.cross_attention_p2p(q, kc, vc, f, heads, prompts=2))
        byt = 2.0 * B * f * hw * C * q.element_size()
        res.append(dict(kernel="cross_attn", hw=hw, d=d, ms=t * 1e3, gbps=byt / t / 1e9))
        k = torch.randn_like(q)
        v = torch.randn_like(q)
        t = timeit(lambda: ops.temporal_attention_p2p(q, k, v, f, heads, prompts=2, self_replace=True))
        byt = 4.0 * B * f * hw * C * q.element_size()
        res.append(dict(kernel="temporal_attn", hw=hw, d=d, ms=t * 1e3, gbps=byt / t / 1e9))
    for r in res:
        print(json.dumps(r))


if __name__ == "__main__":
    main()
