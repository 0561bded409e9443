"""Run only one K10 projection N times (a rocprofv3 --pmc target).
usage: python tools/gemm_only.py plain|geglu|residual M K N [REPS]
  plain: alpha (x @ W^T + b); residual: r + x @ W^T + b; geglu: GEGLU(x @ W^T + b), W with N rows
  (interleaved as the UNet passes it).  At K = 320 and M = B f 4096 these are the K10s stream shapes."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "video-p2p_amd"))
from vp2p import ops  # noqa: E402

kind = sys.argv[1]
M, K, N = (int(v) for v in sys.argv[2:5])
reps = int(sys.argv[5]) if len(sys.argv) > 5 else 5
g = torch.Generator(device="cuda").manual_seed(0)
x = torch.randn(M, K, device="cuda", generator=g).bfloat16()
w = (torch.randn(N, K, device="cuda", generator=g) * 0.05).bfloat16()
b = (torch.randn(N, device="cuda", generator=g) * 0.1).bfloat16()
torch.set_grad_enabled(False)
if kind == "geglu":
    wi, bi = ops.geglu_interleave(w, b)
    fn = lambda: ops.linear_geglu(x, wi, bi)  # noqa: E731
elif kind == "residual":
    r = torch.randn(M, N, device="cuda", generator=g).bfloat16()
    fn = lambda: ops.linear_residual(x, w, b, r)  # noqa: E731
elif kind == "plain":
    fn = lambda: ops.linear_k10(x, w, b)  # noqa: E731
else:
    raise SystemExit(f"unknown kind {kind!r}")
for _ in range(reps):
    fn()
torch.cuda.synchronize()
print("done")
