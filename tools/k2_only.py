"""Runs K2 (cross-attention + fused P2P refine/reweight edit, cond + uncond halves) at one edit
shape N times, for PMC passes: python tools/k2_only.py [N] [hw] [C] [step]
(step < 10: an edit launch; step >= 10: the plain/LocalBlend-free launch of the later steps)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "video-p2p_amd"))
sys.path.insert(0, ROOT)
import vp2p  # noqa: E402
from vp2p import ops  # noqa: E402
from vp2p.tokenizer import SyntheticCLIPTokenizer  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    hw = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    C = int(sys.argv[3]) if len(sys.argv) > 3 else 320
    step = int(sys.argv[4]) if len(sys.argv) > 4 else 3
    prompts, swap, blend, eq, cross, self_ = __import__("bench").RABBIT
    ctrl = vp2p.make_controller(prompts, swap, {"default_": cross}, self_, blend, eq,
                                tokenizer=SyntheticCLIPTokenizer(), num_steps=50)
    plan = ctrl.plan("cuda")
    B, f, heads = 4, 8, 8
    g = torch.Generator(device="cuda").manual_seed(0)
    q = torch.randn(B * f, hw, C, device="cuda", dtype=torch.bfloat16, generator=g)
    k = torch.randn(B, 77, C, device="cuda", dtype=torch.bfloat16, generator=g)
    v = torch.randn(B, 77, C, device="cuda", dtype=torch.bfloat16, generator=g)
    for _ in range(n):
        ops.cross_attention_p2p(q, k, v, f, heads, plan=plan, step=step, edit=step < 10)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
