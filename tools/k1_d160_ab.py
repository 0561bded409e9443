"""K1 at d = 160 (the res-16 and res-8 FrameAttention of SD-1.5: C 1280, 8 heads) and d = 80 (res-32):
timing of the d = 160 kernels selected by VP2P_K1_D160 (1: the resident-K/V kernel, the product form;
0: the one-set kernel), each launch right after its q is rewritten (as by the to_q projection in the
edit), median of reps by HIP events; outputs compared with the first variant.
    python tools/k1_d160_ab.py OUT.jsonl"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "video-p2p_amd"))
from vp2p import ops  # noqa: E402

VARIANTS = os.environ.get("K1AB_VARIANTS", "1,0").split(",")


def main():
    out_path = sys.argv[1] if len(sys.argv) > 1 else "k1_d160_ab.jsonl"
    B, f, heads, reps = 4, 8, 8, 40
    g = torch.Generator(device="cuda").manual_seed(0)
    lines = []
    for hw, C in ((256, 1280), (64, 1280), (1024, 640)):
        d = C // heads
        q = (torch.randn(B * f, hw, C, device="cuda", generator=g) * 0.3).to(torch.bfloat16)
        kv = (torch.randn(B, hw, 2 * C, device="cuda", generator=g) * 0.3).to(torch.bfloat16)
        k, v = kv[..., :C], kv[..., C:]
        zero = torch.zeros((), device="cuda", dtype=torch.bfloat16)
        flops = 4.0 * B * f * hw * hw * C
        res, outs = {}, {}
        for var in VARIANTS + VARIANTS:
            if d != 160 and var != VARIANTS[0]:
                continue
            os.environ["VP2P_K1_D160"] = var
            ts = []
            for _ in range(reps):
                q.add_(zero)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                o = ops.frame_attention(q, k, v, f, heads)
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) * 1e3)
            res.setdefault(var, []).append(sorted(ts)[len(ts) // 2])
            outs[var] = o.clone()
        for var, us in res.items():
            dd = {"hw": hw, "C": C, "d": d, "variant": var, "us": min(us), "tflops": flops / min(us) / 1e6,
                  "frac_2500": flops / min(us) / 1e6 / 2500,
                  "max_abs_diff_vs_first": float((outs[var].float() - outs[VARIANTS[0]].float()).abs().max())}
            print(json.dumps(dd), flush=True)
            lines.append(dd)
    os.environ.pop("VP2P_K1_D160", None)
    with open(out_path, "w") as fh:
        for dd in lines:
            fh.write(json.dumps(dd) + "\n")


if __name__ == "__main__":
    main()
