"""attn_temp's output projection + the block's last residual add (attention.py:268), per UNet level
(B*f = 32, 512^2): hipBLASLt F.linear + a torch add vs K10's GEMM core with the add in its epilogue
(ops.linear_residual).  Prints one JSON line per shape with both times and the max |diff|."""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "video-p2p_amd"))
from vp2p import ops  # noqa: E402


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n


torch.manual_seed(0)
for M, C in ((131072, 320), (32768, 640), (8192, 1280), (2048, 1280)):
    x = torch.randn(32, M // 32, C, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(C, C, device="cuda", dtype=torch.bfloat16) * 0.05
    b = torch.randn(C, device="cuda", dtype=torch.bfloat16) * 0.1
    r = torch.randn(32, M // 32, C, device="cuda", dtype=torch.bfloat16)
    row = {"M": M, "K": C, "N": C}
    t_lib = timeit(lambda: F.linear(x, w, b) + r)
    row["hipblaslt_plus_add_ms"] = round(t_lib, 4)
    if ops.linear_residual_supported(x, w, r):
        t_k = timeit(lambda: ops.linear_residual(x, w, b, r))
        d = (ops.linear_residual(x, w, b, r).float() - (F.linear(x, w, b) + r).float()).abs().max().item()
        row.update({"k10_res_ms": round(t_k, 4), "max_abs_diff": d})
    print(json.dumps(row), flush=True)
