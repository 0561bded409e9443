"""K10's one-pass tile configurations on the projection shapes hipBLASLt keeps (res-16 / res-32 rows of
an 8-frame B4 edit) against hipBLASLt; one JSON line per shape with an output checksum, so lab builds
(tools/lab_build.sh NAME conv -DVP2P_K10_FORCE_CF=c) compare bit for bit.
usage: python tools/k10_linear_cf_bench.py OUT.jsonl   (VP2P_LIB selects the build)"""
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
    for _ in range(7):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(n):
            fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e) / n)
    return sorted(ts)[3]


lib = os.path.basename(os.environ.get("VP2P_LIB", "libvp2p_hip.so"))
SHAPES = [(8192, C * a, C * b) for C in (1280,) for a, b in ((1, 1), (1, 2), (1, 3), (4, 1))]
SHAPES += [(32768, C * a, C * b) for C in (640,) for a, b in ((1, 1), (1, 2), (1, 3), (4, 1))]
SHAPES += [(131072, 320, 960), (131072, 1280, 320)]
g = torch.Generator(device="cuda").manual_seed(0)
with torch.no_grad(), open(sys.argv[1], "a") as fh:
    for M, K, N in SHAPES:
        x = torch.randn(M, K, device="cuda", generator=g).bfloat16()
        w = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).bfloat16()
        b = (torch.randn(N, device="cuda", generator=g) * 0.1).bfloat16()
        y = ops.linear_k10(x, w, b)
        t = timeit(lambda: ops.linear_k10(x, w, b))
        tl = timeit(lambda: F.linear(x, w, b))
        r = dict(lib=lib, M=M, K=K, N=N, us=round(t * 1e3, 2), hipblaslt_us=round(tl * 1e3, 2),
                 tflops=round(2.0 * M * K * N / t / 1e9, 1), sum=y.float().abs().sum().item())
        print(json.dumps(r), flush=True)
        fh.write(json.dumps(r) + "\n")
