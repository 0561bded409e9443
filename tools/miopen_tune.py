"""Tune MIOpen's convolution kernels for the UNet3D shapes the pipeline runs, into an in-tree
user perf/find database that bench.py and the pipeline then reuse (no tuning at run time).

Run on the MI355X with the database directory and search mode in the environment, e.g.
  MIOPEN_USER_DB_PATH=$PWD/miopen_db MIOPEN_FIND_ENFORCE=3 python tools/miopen_tune.py
It drives the convolutions of one UNet forward at every batch the pipeline uses (edit: 4 =
2 prompts x CFG; inversion: 1; null-text: 1 and 2 with backward) for --frames frames at 512^2,
with torch.backends.cudnn.benchmark on (miopenFind per shape; FIND_ENFORCE=3 makes it tune
every solver's kernel parameters and store the winners).
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "video-p2p_amd"))
from vp2p.unet3d import UNet3DConditionModel, init_random_  # noqa: E402


def drive(frames, batches, backward):
    """One UNet forward (and backward w.r.t. the embedding for the batches in ``backward``) at every
    batch in ``batches``: every conv and GEMM shape the pipeline runs at ``frames`` frames, 512^2."""
    dev = torch.device("cuda")
    unet = init_random_(UNet3DConditionModel(), seed=0).to(dev, torch.bfloat16).to(memory_format=torch.channels_last)
    unet.eval()
    unet.requires_grad_(False)   # null-text differentiates w.r.t. the embedding only
    bwd = {int(b) for b in backward.split(",") if b}
    for B in [int(b) for b in batches.split(",")]:
        t0 = time.time()
        x = torch.randn(B, 4, frames, 64, 64, device=dev)
        ctx = torch.randn(B, 77, 768, device=dev, requires_grad=B in bwd)
        with torch.set_grad_enabled(B in bwd):
            out = unet(x, 981, ctx).sample
            if B in bwd:
                out.float().square().mean().backward()
        torch.cuda.synchronize()
        print(f"batch {B}{' +bwd' if B in bwd else ''}: {time.time() - t0:.1f} s", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=8)
    ap.add_argument("--batches", default="4,1,2")
    ap.add_argument("--backward", default="1,2", help="batches also run through backward (null-text)")
    args = ap.parse_args()
    torch.backends.cudnn.benchmark = True
    drive(args.frames, args.batches, args.backward)


if __name__ == "__main__":
    main()
