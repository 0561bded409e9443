"""K2 (hooked cross-attention + fused P2P edit) timing at the edit's shapes, one JSON line per case.

  python tools/k2_bench.py [--iters 50]

Cases: the rabbit edit (AttentionRefine + Reweight) at B = 4 (2 prompts x CFG), 8 frames:
res-64 (4096 tokens, C 320, d 40) edit on / off, res-16 with the LocalBlend sum (256 tokens, C 1280),
res-32 (1024, C 640).  HBM bytes = Q in + O out + K/V once per batch row (bf16), as bench.py counts.
Also writes the output checksum so two kernels' results can be compared.
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "video-p2p_amd"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--producer", type=int, default=0,
                    help="1: rewrite q in place before each launch (its projection writes it right before K2 in "
                         "the edit) and time each launch alone by events")
    args = ap.parse_args()
    import vp2p
    from vp2p import ops
    from vp2p.tokenizer import SyntheticCLIPTokenizer
    prompts, swap, blend, eq, cross, self_ = __import__("bench").RABBIT
    ctrl = vp2p.make_controller(prompts, swap, {"default_": cross}, self_, blend, eq,
                                tokenizer=SyntheticCLIPTokenizer(), num_steps=50)
    plan = ctrl.plan("cuda")
    B, f, heads = 4, 8, 8
    cases = [("res64_edit", 4096, 320, 3, False), ("res64_noedit", 4096, 320, 30, False),
             ("res32_edit", 1024, 640, 3, False), ("res16_lb", 256, 1280, 30, True),
             ("res16_edit_lb", 256, 1280, 3, True)]
    for name, hw, C, step, lb in cases:
        g = torch.Generator(device="cuda").manual_seed(0)
        q = torch.randn(B * f, hw, C, device="cuda", dtype=torch.bfloat16, generator=g)
        k = torch.randn(B, 77, C, device="cuda", dtype=torch.bfloat16, generator=g)
        v = torch.randn(B, 77, C, device="cuda", dtype=torch.bfloat16, generator=g)
        acc = torch.zeros(2, f, hw, device="cuda") if lb else None
        out = torch.empty_like(q)
        edit = step < 10
        run = lambda: ops.cross_attention_p2p(q, k, v, f, heads, plan=plan, step=step, edit=edit,  # noqa: E731
                                              lb_acc=acc, out=out)
        for _ in range(3):
            run()
        if args.producer:
            zero = torch.zeros((), device="cuda", dtype=torch.bfloat16)
            ts = []
            for _ in range(args.iters):
                q.add_(zero)
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                run()
                e.record()
                e.synchronize()
                ts.append(s.elapsed_time(e) * 1e3)
            us = sorted(ts)[len(ts) // 2]
        else:
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(args.iters):
                run()
            e.record()
            e.synchronize()
            us = s.elapsed_time(e) / args.iters * 1e3
        nbytes = 2 * (2 * B * f * hw * C + 2 * B * 77 * C)
        print(json.dumps({"case": name, "us": round(us, 2),
                          "gbs": round(nbytes / us / 1e3, 1), "frac_8tbs": round(nbytes / us / 1e3 / 8000, 4),
                          "checksum": float(out.float().abs().sum()),
                          "lb_checksum": None if acc is None else float(acc.sum())}), flush=True)


if __name__ == "__main__":
    main()
