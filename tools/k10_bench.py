"""K10 (conv / GEMM core) timing at the edit's shapes (B*f = 32, 512^2): 3x3 convs, 1x1 projections,
the GEGLU projection and the split-K small shapes; prints TF/s and an output checksum so builds can be
compared bit for bit.  usage: python tools/k10_bench.py OUT.jsonl   (library from VP2P_LIB)"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "video-p2p_amd"))
from vp2p import ops  # noqa: E402


def timeit(fn, n=10):
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
        ts.append(s.elapsed_time(e) / n)
    return sorted(ts)[2]


lib = os.path.basename(os.environ.get("VP2P_LIB", "libvp2p_hip.so"))
g = torch.Generator(device="cuda").manual_seed(0)
rows = []
# 3x3 convs: (n, cin, h, cout, stride, residual)
for n, cin, h, cout, st, res in ((32, 320, 64, 320, 1, True), (32, 640, 64, 320, 1, True), (32, 640, 32, 640, 1, True),
                                 (32, 1280, 16, 1280, 1, True), (32, 2560, 16, 1280, 1, False), (32, 1920, 16, 1280, 1, False),
                                 (32, 1280, 8, 1280, 1, False),
                                 (32, 320, 64, 320, 2, False), (32, 2560, 8, 1280, 1, True)):
    x = torch.randn(n, cin, h, h, device="cuda", generator=g).bfloat16().to(memory_format=torch.channels_last)
    w = (torch.randn(cout, cin, 3, 3, device="cuda", generator=g) * 0.02).bfloat16().to(memory_format=torch.channels_last)
    b = (torch.randn(cout, device="cuda", generator=g) * 0.1).bfloat16()
    ho = (h + 2 - 3) // st + 1
    r = torch.randn(n, cout, ho, ho, device="cuda", generator=g).bfloat16().to(memory_format=torch.channels_last) if res else None
    y = ops.conv2d(x, w, b, st, 1, residual=r)
    t = timeit(lambda: ops.conv2d(x, w, b, st, 1, residual=r))
    fl = 2.0 * n * ho * ho * cout * 9 * cin
    rows.append(dict(lib=lib, op="conv3x3", shape=[n, cin, h, cout, st], ms=round(t, 4), tflops=round(fl / t / 1e9, 1),
                     sum=y.float().abs().sum().item()))
# 1x1 projections (M, K, N) with a residual, and the GEGLU projection
for M, K, N in ((131072, 320, 320), (131072, 1280, 320), (32768, 640, 640), (8192, 1280, 1280), (2048, 1280, 1280)):
    x = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    w = (torch.randn(N, K, device="cuda", generator=g) * 0.05).bfloat16()
    b = (torch.randn(N, device="cuda", generator=g) * 0.1).bfloat16()
    r = torch.randn(M, N, device="cuda", generator=g).bfloat16()
    x4 = x.view(M, 1, 1, K).permute(0, 3, 1, 2)
    w4 = w.view(N, K, 1, 1)
    r4 = r.view(M, 1, 1, N).permute(0, 3, 1, 2)
    y = ops.conv2d(x4, w4, b, 1, 0, residual=r4)
    t = timeit(lambda: ops.conv2d(x4, w4, b, 1, 0, residual=r4))
    rows.append(dict(lib=lib, op="linear", shape=[M, K, N], ms=round(t, 4), tflops=round(2.0 * M * K * N / t / 1e9, 1),
                     sum=y.float().abs().sum().item()))
for M, K in ((131072, 320), (32768, 640)):
    inner = 4 * K
    x = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    w = (torch.randn(2 * inner, K, device="cuda", generator=g) * 0.05).bfloat16()
    b = (torch.randn(2 * inner, device="cuda", generator=g) * 0.1).bfloat16()
    wi, bi = ops.geglu_interleave(w, b)
    y = ops.linear_geglu(x, wi, bi)
    t = timeit(lambda: ops.linear_geglu(x, wi, bi))
    rows.append(dict(lib=lib, op="geglu", shape=[M, K, 2 * inner], ms=round(t, 4),
                     tflops=round(2.0 * M * K * 2 * inner / t / 1e9, 1), sum=y.float().abs().sum().item()))
with open(sys.argv[1], "a") as fh:
    for r in rows:
        print(json.dumps(r), flush=True)
        fh.write(json.dumps(r) + "\n")
