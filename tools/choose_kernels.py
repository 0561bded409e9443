"""Measure K10 against the library path for every shape the pipeline runs and write the in-tree
choice table ``miopen_db/kernel_choices.json`` that ``vp2p.ops.ConvSelector`` reads (no timing at
run time: every run, box and rank then takes the same kernels and the same numerics).

Run on the MI355X:  python tools/choose_kernels.py [--out miopen_db/kernel_choices.json]
It drives one UNet3D forward (bf16, 512^2) at every (UNet batch, frames-per-rank) the pipeline
uses -- the edit (B 4), the inversion (B 1), the null-text step (B 2), the CFG-split multi-GPU ranks
(B 2 with 8/4/2 frames of an 8-frame clip, 24/12/6 of a 24-frame clip) -- with VP2P_CONV=tune, so
each new shape is timed once (5 launches of each candidate after 2 warm-ups, HIP events).
"""
import argparse
import json
import os
import sys
import time

os.environ["VP2P_CONV"] = "tune"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "video-p2p_amd"))

import torch  # noqa: E402

CASES = [(4, 8), (1, 8), (2, 8), (2, 4), (2, 2), (4, 24), (1, 24), (2, 24), (2, 12), (2, 6),
         (4, 1), (4, 2), (4, 4), (2, 1), (1, 1), (1, 2)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "miopen_db", "kernel_choices.json"))
    ap.add_argument("--cases", default=",".join(f"{b}x{f}" for b, f in CASES))
    args = ap.parse_args()
    t0 = time.time()
    from vp2p import ops
    from vp2p.tuning import use_tuned_libraries
    from vp2p.unet3d import UNet3DConditionModel, init_random_
    use_tuned_libraries()
    import threading

    def beat():          # new conv shapes compile MIOpen kernels for minutes: keep the run visibly alive
        while True:
            time.sleep(30)
            print(f"[choose] ... {len(ops.CONV.choice)} shapes ({time.time() - t0:.0f} s)", flush=True)
    threading.Thread(target=beat, daemon=True).start()
    dev = torch.device("cuda")
    unet = init_random_(UNet3DConditionModel(), seed=0).to(dev, torch.bfloat16).to(memory_format=torch.channels_last)
    unet.eval()
    with torch.no_grad():
        for case in args.cases.split(","):
            B, f = (int(v) for v in case.split("x"))
            x = torch.randn(B, 4, f, 64, 64, device=dev, dtype=torch.bfloat16)
            ctx = torch.randn(B, 77, 768, device=dev, dtype=torch.bfloat16)
            unet(x, 501, ctx)
            torch.cuda.synchronize()
            print(f"[choose] B={B} f={f}: {len(ops.CONV.choice)} shapes so far ({time.time() - t0:.0f} s)", flush=True)
    table = {"how": "tools/choose_kernels.py on an MI355X: per shape, 5 timed launches of K10 vs the library path "
                    "(after 2 warm-ups); true = K10",
             "device": torch.cuda.get_device_name(dev),
             "choices": dict(sorted(ops.CONV.choice.items()))}
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as fh:
        json.dump(table, fh, indent=1)
    k10 = sum(table["choices"].values())
    print(f"wrote {args.out}: {len(table['choices'])} shapes, K10 chosen for {k10}")


if __name__ == "__main__":
    main()
