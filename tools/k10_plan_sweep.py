"""K10 launch-plan sweep at the small-clip shapes: every 3x3 conv of the SD-1.5 UNet at n = 4 f images
(B4 edit of an f-frame clip), timed under each valid VP2P_K10_PLAN="CF,K" (tile configuration, K-split)
and under the library's own choice ("auto"), with the output compared against auto's (one-pass tiles are
bit-equal; K-splits round once from an fp32 sum of slices).
usage: python tools/k10_plan_sweep.py OUT.jsonl [--linear] [frames ...]      (default frames: 1 2 3;
--linear: the 1x1 projections instead, with hipBLASLt as one more row)"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "video-p2p_amd"))
from vp2p import ops  # noqa: E402

PLANS = ["auto"] + [f"{cf},1" for cf in range(5)] + [f"{cf},{k}" for cf in (0, 3, 4) for k in (2, 3, 4, 6, 8)]
# (cin, h, cout, stride, upsample): resnet convs, Downsample2D (stride 2), Upsample3D (x2 nearest on the fly)
SHAPES = [(320, 64, 320, 1, 0), (640, 64, 320, 1, 0), (960, 64, 320, 1, 0),
          (320, 32, 640, 1, 0), (640, 32, 640, 1, 0), (1280, 32, 640, 1, 0), (960, 32, 640, 1, 0),
          (640, 16, 1280, 1, 0), (1280, 16, 1280, 1, 0), (2560, 16, 1280, 1, 0), (1920, 16, 1280, 1, 0),
          (1280, 8, 1280, 1, 0), (2560, 8, 1280, 1, 0),
          (320, 64, 320, 2, 0), (640, 32, 640, 2, 0), (1280, 16, 1280, 2, 0),
          (1280, 16, 1280, 1, 1), (1280, 32, 1280, 1, 1), (640, 64, 640, 1, 1)]


def timeit(fn, n=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    t0 = time.time()
    while time.time() - t0 < 0.05:      # clocks up before the first plan of a shape is timed
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


def set_plan(p):
    if p == "auto":
        os.environ.pop("VP2P_K10_PLAN", None)
    else:
        os.environ["VP2P_K10_PLAN"] = p
    ops._CONV_WS.clear()


def sweep_linear(fh, f, g):
    """the projections (x W^T + b, K10's 1x1 core) at the f-frame clip's row counts, each plan and
    hipBLASLt ("library", F.linear)"""
    for hw, K, N in LSHAPES:
        M = 4 * f * hw
        x = torch.randn(M, K, device="cuda", generator=g).bfloat16()
        w = (torch.randn(N, K, device="cuda", generator=g) * 0.05).bfloat16()
        b = (torch.randn(N, device="cuda", generator=g) * 0.1).bfloat16()
        fl = 2.0 * M * K * N
        ref = None
        for p in PLANS + ["library"]:
            set_plan("auto" if p == "library" else p)
            fn = (lambda: torch.nn.functional.linear(x, w, b)) if p == "library" else (lambda: ops.linear_k10(x, w, b))
            y = fn()
            if ref is None:
                ref = y
            t = timeit(fn)
            d = (y.float() - ref.float()).abs().max().item()
            row = dict(frames=f, linear=[M, K, N], plan=p, ms=round(t, 4), tflops=round(fl / t / 1e9, 1),
                       equal=bool(torch.equal(y, ref)), maxdiff=d)
            print(json.dumps(row), flush=True)
            fh.write(json.dumps(row) + "\n")
        set_plan("auto")


# (pixels per image, K, N) of the transformer / resnet projections at res-32 / 16 / 8 and the res-64 FF out
LSHAPES = [(1024, 640, 640), (1024, 2560, 640), (1024, 1280, 640), (1024, 960, 640),
           (256, 1280, 1280), (256, 5120, 1280), (256, 2560, 1280), (256, 1920, 1280), (64, 1280, 1280),
           (4096, 1280, 320), (4096, 640, 320), (4096, 960, 320)]


def main():
    out = sys.argv[1]
    args = sys.argv[2:]
    linear = "--linear" in args
    frames = [int(f) for f in args if f != "--linear"] or [1, 2, 3]
    g = torch.Generator(device="cuda").manual_seed(0)
    with open(out, "a") as fh:
        if linear:
            for f in frames:
                sweep_linear(fh, f, g)
            return
        for f in frames:
            n = 4 * f
            for cin, h, cout, st, up in SHAPES:
                hs = h // 2 if up else h        # stored input of the upsampling conv
                x = torch.randn(n, cin, hs, hs, device="cuda", generator=g).bfloat16().to(memory_format=torch.channels_last)
                w = (torch.randn(cout, cin, 3, 3, device="cuda", generator=g) * 0.02).bfloat16().to(
                    memory_format=torch.channels_last)
                b = (torch.randn(cout, device="cuda", generator=g) * 0.1).bfloat16()
                ho = (h + 2 - 3) // st + 1
                fl = 2.0 * n * ho * ho * cout * 9 * cin
                ref = None
                for p in PLANS:
                    set_plan(p)
                    fn = lambda: ops.conv2d(x, w, b, st, 1, upsample=bool(up))  # noqa: E731
                    y = fn()
                    if ref is None:
                        ref = y
                    t = timeit(fn)
                    d = (y.float() - ref.float()).abs().max().item()
                    row = dict(frames=f, shape=[n, cin, h, cout, st, up], plan=p, ms=round(t, 4),
                               tflops=round(fl / t / 1e9, 1), equal=bool(torch.equal(y, ref)), maxdiff=d)
                    print(json.dumps(row), flush=True)
                    fh.write(json.dumps(row) + "\n")
                set_plan("auto")


if __name__ == "__main__":
    main()
