"""FeedForward GEGLU projection at the UNet's shapes (B*f = 32, 512^2): hipBLASLt GEMM + K9 vs the
K10 GEMM with the GEGLU epilogue; also plain K10 1x1 vs hipBLASLt for the same GEMM."""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "video-p2p_amd"))
from vp2p import ops  # noqa: E402


def timeit(fn, n=10):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n


for M, K in ((131072, 320), (32768, 640), (8192, 1280), (2048, 1280)):
    inner = 4 * K
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(2 * inner, K, device="cuda", dtype=torch.bfloat16) * 0.05
    b = torch.zeros(2 * inner, device="cuda", dtype=torch.bfloat16)
    wi, bi = ops.geglu_interleave(w, b)
    t_gemm = timeit(lambda: F.linear(x, w, b))
    h = F.linear(x, w, b)
    t_geglu = timeit(lambda: ops.geglu(h))
    t_fused = timeit(lambda: ops.linear_geglu(x, wi, bi))
    fl = 2.0 * M * K * 2 * inner
    print(json.dumps({"M": M, "K": K, "N": 2 * inner, "gemm_ms": round(t_gemm, 4), "gemm_tflops": round(fl / t_gemm / 1e9, 1),
                      "geglu_ms": round(t_geglu, 4), "fused_ms": round(t_fused, 4),
                      "fused_tflops": round(fl / t_fused / 1e9, 1)}), flush=True)
