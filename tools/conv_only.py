"""Run only one K10 3x3 conv shape N times (a rocprofv3 --pmc target).
usage: python tools/conv_only.py N CIN H COUT [REPS]   (B*f = N images, channels-last bf16, residual)"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "video-p2p_amd"))
from vp2p import ops  # noqa: E402

n, cin, h, cout = (int(v) for v in sys.argv[1:5])
reps = int(sys.argv[5]) if len(sys.argv) > 5 else 5
x = torch.randn(n, cin, h, h, device="cuda").bfloat16().to(memory_format=torch.channels_last)
w = (torch.randn(cout, cin, 3, 3, device="cuda") * 0.02).bfloat16().to(memory_format=torch.channels_last)
b = torch.zeros(cout, device="cuda").bfloat16()
r = torch.randn(n, cout, h, h, device="cuda").bfloat16().to(memory_format=torch.channels_last)
for _ in range(reps):
    ops.conv2d(x, w, b, 1, 1, residual=r)
torch.cuda.synchronize()
print("done")
