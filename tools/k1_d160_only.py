"""Runs K1 at the res-16 d = 160 shape (B4 f8, 256 tokens, C 1280) N times, for rocprofv3 passes.
python tools/k1_d160_only.py [N] [hw]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "video-p2p_amd"))
from vp2p import ops  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 5
hw = int(sys.argv[2]) if len(sys.argv) > 2 else 256
B, f, heads, C = 4, 8, 8, 1280
g = torch.Generator(device="cuda").manual_seed(0)
q = (torch.randn(B * f, hw, C, device="cuda", generator=g) * 0.3).to(torch.bfloat16)
kv = (torch.randn(B, hw, 2 * C, device="cuda", generator=g) * 0.3).to(torch.bfloat16)
for _ in range(n):
    o = ops.frame_attention(q, kv[..., :C], kv[..., C:], f, heads)
torch.cuda.synchronize()
print("k1_d160_only done", float(o.float().abs().sum()))
