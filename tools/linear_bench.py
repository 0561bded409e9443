"""The UNet's projection GEMMs (B*f = 32, 512^2): hipBLASLt (F.linear) vs K10's GEMM core."""
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


shapes = []
for M, C in ((131072, 320), (32768, 640), (8192, 1280), (2048, 1280)):
    shapes += [(M, C, C), (M, C, 3 * C), (M, 4 * C, C), (M // 8, C, 2 * C)]
for M, K, N in shapes:
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.05
    b = torch.zeros(N, device="cuda", dtype=torch.bfloat16)
    r = torch.zeros(M, N, device="cuda", dtype=torch.bfloat16)
    t_lib = timeit(lambda: F.linear(x, w, b))
    row = {"M": M, "K": K, "N": N, "hipblaslt_ms": round(t_lib, 4),
           "hipblaslt_tflops": round(2.0 * M * K * N / t_lib / 1e9, 1)}
    if ops.linear_residual_supported(x, w, r):
        t_k = timeit(lambda: ops.linear_residual(x, w, b, r))
        row.update({"k10_res_ms": round(t_k, 4), "k10_tflops": round(2.0 * M * K * N / t_k / 1e9, 1)})
    print(json.dumps(row), flush=True)
