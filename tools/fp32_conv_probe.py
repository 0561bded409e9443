"""fp32 MIOpen convolutions at the UNet's 3x3 shapes for image batches N (2 prompts x CFG x frames):
per shape and N, the time of F.conv2d on channels-last fp32 -- where the fp32 edit's time goes as the
frame count grows.   usage: python tools/fp32_conv_probe.py OUT.jsonl N [N ...]"""
import json
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "video-p2p_amd"))
from vp2p.tuning import use_tuned_libraries  # noqa: E402

use_tuned_libraries()
SHAPES = ((64, 320, 320), (32, 640, 640), (16, 1280, 1280), (8, 1280, 1280), (64, 640, 320), (32, 1280, 640))
out = open(sys.argv[1], "a")
for n in [int(a) for a in sys.argv[2:]]:
    for h, cin, cout in SHAPES:
        x = torch.randn(n, cin, h, h, device="cuda").to(memory_format=torch.channels_last)
        w = (torch.randn(cout, cin, 3, 3, device="cuda") * 0.02).to(memory_format=torch.channels_last)
        t0 = time.time()
        F.conv2d(x, w, None, 1, 1)
        torch.cuda.synchronize()
        first = time.time() - t0
        t0 = time.time()
        for _ in range(3):
            F.conv2d(x, w, None, 1, 1)
        torch.cuda.synchronize()
        ms = (time.time() - t0) / 3 * 1e3
        r = dict(n=n, h=h, cin=cin, cout=cout, first_s=round(first, 3), ms=round(ms, 3),
                 tflops=round(2 * n * h * h * cin * cout * 9 / ms / 1e9, 1))
        print(json.dumps(r), flush=True)
        out.write(json.dumps(r) + "\n")
        del x, w
