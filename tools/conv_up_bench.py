"""Time K10's fused x2-upsample 3x3 convs (Upsample3D, resnet.py:79-99) at the edit's shapes and check
them against F.interpolate + conv2d (fp32).  usage: python tools/conv_up_bench.py OUT.jsonl
(the library comes from VP2P_LIB, so two builds can be compared)."""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "video-p2p_amd"))
from vp2p import ops  # noqa: E402

out = sys.argv[1]
rows = []
g = torch.Generator(device="cuda").manual_seed(0)
for n, c, h in ((32, 1280, 8), (32, 1280, 16), (32, 640, 32)):
    x = torch.randn(n, c, h, h, device="cuda", generator=g).bfloat16().to(memory_format=torch.channels_last)
    w = (torch.randn(c, c, 3, 3, device="cuda", generator=g) * 0.02).bfloat16().to(memory_format=torch.channels_last)
    b = (torch.randn(c, device="cuda", generator=g) * 0.1).bfloat16()
    y = ops.conv2d(x, w, b, 1, 1, upsample=True)
    ref = F.conv2d(F.interpolate(x.float(), scale_factor=2.0, mode="nearest"), w.float(), b.float(), 1, 1)
    err = ((y.float() - ref).abs().max() / ref.abs().max()).item()
    for _ in range(3):
        ops.conv2d(x, w, b, 1, 1, upsample=True)
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(10):
            ops.conv2d(x, w, b, 1, 1, upsample=True)
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e) / 10)
    ts.sort()
    fl = 2.0 * n * (2 * h) ** 2 * c * 9 * c
    r = dict(lib=os.path.basename(os.environ.get("VP2P_LIB", "libvp2p_hip.so")), n=n, c=c, h_out=2 * h,
             ms=round(ts[2], 4), tflops=round(fl / ts[2] / 1e9, 1), rel_err=err, sum=y.float().abs().sum().item())
    print(json.dumps(r), flush=True)
    rows.append(r)
with open(out, "a") as fh:
    for r in rows:
        fh.write(json.dumps(r) + "\n")
