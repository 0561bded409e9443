"""Run only K1 (res-64 FrameAttention, B=4 f=8 d=40 bf16, pre-scaled q as in the UNet) N times: a target
for rocprofv3 --pmc."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "video-p2p_amd"))
from vp2p import ops  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10
hw, C, B, f, heads = 4096, 320, 4, 8, 8
q = (torch.randn(B * f, hw, C, device="cuda") * ops.frame_query_scale(C // heads)).bfloat16()
k0 = torch.randn(B, hw, C, device="cuda", dtype=torch.bfloat16)
v0 = torch.randn(B, hw, C, device="cuda", dtype=torch.bfloat16)
for _ in range(n):
    ops.frame_attention(q, k0, v0, f, heads, q_prescaled=True)
torch.cuda.synchronize()
print("done")
