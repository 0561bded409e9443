"""Run only the fused K10 GEGLU projection N times (a rocprofv3 --pmc target).
usage: python tools/geglu_only.py M K INNER [REPS]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "video-p2p_amd"))
from vp2p import ops  # noqa: E402

M, K, inner = (int(v) for v in sys.argv[1:4])
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 5
x = torch.randn(M, K, device="cuda").bfloat16()
w = (torch.randn(2 * inner, K, device="cuda") * 0.05).bfloat16()
b = (torch.randn(2 * inner, device="cuda") * 0.1).bfloat16()
wi, bi = ops.geglu_interleave(w, b)
for _ in range(reps):
    ops.linear_geglu(x, wi, bi)
torch.cuda.synchronize()
print("done")
