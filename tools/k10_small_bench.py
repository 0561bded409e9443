"""K10 at the small-clip shapes (a 1- or 2-frame B4 edit: n = B*f = 4 / 8 images of 64^2 latents):
the 3x3 convs of every resolution and the plain projections, K10 vs the library (MIOpen conv /
hipBLASLt GEMM) on the same inputs; prints one JSON line per shape with an output checksum so that
builds can be compared bit for bit.   usage: python tools/k10_small_bench.py OUT.jsonl  (VP2P_LIB)"""
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
CONVS = ((64, 320, 320), (64, 640, 320), (64, 960, 320), (32, 320, 640), (32, 640, 640), (32, 1280, 640),
         (16, 640, 1280), (16, 1280, 1280), (16, 2560, 1280), (8, 1280, 1280), (8, 2560, 1280))
with torch.no_grad():
    for n in (4, 8):
        for h, cin, cout in CONVS:
            x = torch.randn(n, cin, h, h, device="cuda", generator=g).bfloat16().to(memory_format=torch.channels_last)
            w = (torch.randn(cout, cin, 3, 3, device="cuda", generator=g) * 0.02).bfloat16()
            w = w.to(memory_format=torch.channels_last)
            b = (torch.randn(cout, device="cuda", generator=g) * 0.1).bfloat16()
            y = ops.conv2d(x, w, b, 1, 1)
            t = timeit(lambda: ops.conv2d(x, w, b, 1, 1))
            tl = timeit(lambda: F.conv2d(x, w, b, 1, 1))
            fl = 2.0 * n * h * h * cout * 9 * cin
            rows.append(dict(lib=lib, op="conv3x3", shape=[n, cin, h, cout], ms=round(t, 4), lib_ms=round(tl, 4),
                             tflops=round(fl / t / 1e9, 1), sum=y.float().abs().sum().item()))
        for hw, K, N in ((4096, 320, 320), (1024, 640, 640), (256, 1280, 1280), (64, 1280, 1280)):
            M = n * hw
            x = torch.randn(M, K, device="cuda", generator=g).bfloat16()
            w = (torch.randn(N, K, device="cuda", generator=g) * 0.05).bfloat16()
            b = (torch.randn(N, device="cuda", generator=g) * 0.1).bfloat16()
            y = ops.linear_k10(x, w, b)
            t = timeit(lambda: ops.linear_k10(x, w, b))
            tl = timeit(lambda: F.linear(x, w, b))
            rows.append(dict(lib=lib, op="linear", shape=[M, K, N], ms=round(t, 4), lib_ms=round(tl, 4),
                             tflops=round(2.0 * M * K * N / t / 1e9, 1), sum=y.float().abs().sum().item()))
with open(sys.argv[1], "a") as fh:
    for r in rows:
        print(json.dumps(r), flush=True)
        fh.write(json.dumps(r) + "\n")
