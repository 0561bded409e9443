"""Host cost per call of the library convs left on the UNet path (conv_in 4 -> 320, conv_out 320 -> 4,
MIOpen) and of a hipBLASLt linear, at the 8-frame edit batch (32 images) and a 2-frame rank slice
(4 images): wall time of 20 back-to-back calls without a sync, then with the sync.
usage: python tools/conv_host_cost.py OUT.jsonl"""
import json
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "video-p2p_amd"))
from vp2p.tuning import use_tuned_libraries  # noqa: E402

use_tuned_libraries()
rows = []
for n in (32, 4):
    for name, cin, cout in (("conv_in", 4, 320), ("conv_out", 320, 4)):
        x = torch.randn(n, cin, 64, 64, device="cuda").bfloat16().to(memory_format=torch.channels_last)
        w = torch.randn(cout, cin, 3, 3, device="cuda").bfloat16().to(memory_format=torch.channels_last)
        b = torch.randn(cout, device="cuda").bfloat16()
        for _ in range(3):
            F.conv2d(x, w, b, 1, 1)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            F.conv2d(x, w, b, 1, 1)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        rows.append(dict(op=name, images=n, host_us_per_call=round((t1 - t0) / 20 * 1e6, 1),
                         wall_us_per_call=round((t2 - t0) / 20 * 1e6, 1)))
    x = torch.randn(n * 4096, 320, device="cuda").bfloat16()
    w = torch.randn(320, 320, device="cuda").bfloat16()
    for _ in range(3):
        F.linear(x, w)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        F.linear(x, w)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    rows.append(dict(op="linear 320x320", images=n, host_us_per_call=round((t1 - t0) / 20 * 1e6, 1),
                     wall_us_per_call=round((t2 - t0) / 20 * 1e6, 1)))
with open(sys.argv[1], "a") as fh:
    for r in rows:
        print(json.dumps(r))
        fh.write(json.dumps(r) + "\n")
