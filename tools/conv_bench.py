"""Per-shape timing of the UNet3D's convolutions (B*f = 32, 512^2) on the library path, to size the
conv roofline gap.  Collects every conv call of one forward (hooks), then times each unique shape.
usage: python tools/conv_bench.py [--batch 4] [--frames 8]"""
import argparse
import collections
import json
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "video-p2p_amd"))
from vp2p.tuning import use_tuned_libraries  # noqa: E402

use_tuned_libraries()
from vp2p import ops  # noqa: E402
from vp2p.unet3d import UNet3DConditionModel, init_random_  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--frames", type=int, default=8)
    args = ap.parse_args()
    dev = torch.device("cuda")
    unet = init_random_(UNet3DConditionModel(), seed=0).to(dev, torch.bfloat16).to(memory_format=torch.channels_last)
    unet.eval()
    shapes = collections.Counter()

    def hook(mod, inp, out):
        x = inp[0]
        shapes[(tuple(x.shape), mod.out_channels, mod.kernel_size[0], mod.stride[0], mod.padding[0])] += 1

    hs = [m.register_forward_hook(hook) for m in unet.modules() if isinstance(m, torch.nn.Conv2d)
          and m.kernel_size[0] == 3 or (isinstance(m, torch.nn.Conv2d) and type(m).__name__ == "InflatedConv3d")]
    with torch.no_grad():
        unet(torch.randn(args.batch, 4, args.frames, 64, 64, device=dev), 981,
             torch.randn(args.batch, 77, 768, device=dev))
    for h in hs:
        h.remove()
    total_ms, total_fl, total_best = 0.0, 0.0, 0.0
    rows = []
    for (xs, co, k, st, pad), n in sorted(shapes.items(), key=lambda t: -t[1]):
        x = torch.randn(xs, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        w = (torch.randn(co, xs[1], k, k, device=dev, dtype=torch.bfloat16) * 0.02).contiguous(memory_format=torch.channels_last)
        b = torch.zeros(co, device=dev, dtype=torch.bfloat16)
        for _ in range(3):
            y = F.conv2d(x, w, b, st, pad)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(10):
            y = F.conv2d(x, w, b, st, pad)
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / 10
        fl = 2.0 * y.numel() * xs[1] * k * k
        row = {"x": xs, "cout": co, "k": k, "stride": st, "calls": n, "ms": round(ms, 4),
               "tflops": round(fl / ms / 1e9, 1)}
        best = ms
        if ops.conv2d_supported(x, w, st, pad):
            y2 = ops.conv2d(x, w, b, st, pad)
            err = (y2.float() - y.float()).abs().max().item() / max(y.float().abs().max().item(), 1e-6)
            for _ in range(3):
                ops.conv2d(x, w, b, st, pad)
            s.record()
            for _ in range(10):
                ops.conv2d(x, w, b, st, pad)
            e.record()
            torch.cuda.synchronize()
            ms2 = s.elapsed_time(e) / 10
            row.update({"k10_ms": round(ms2, 4), "k10_tflops": round(fl / ms2 / 1e9, 1), "k10_rel_err": round(err, 5)})
            best = min(ms, ms2)
        total_ms += ms * n
        total_best += best * n
        total_fl += fl * n
        rows.append(row)
        print(json.dumps(rows[-1]), flush=True)
    print(json.dumps({"total_ms_per_forward": round(total_ms, 3), "total_tflop": round(total_fl / 1e12, 3),
                      "avg_tflops": round(total_fl / total_ms / 1e9, 1),
                      "best_of_both_ms_per_forward": round(total_best, 3)}))


if __name__ == "__main__":
    main()
