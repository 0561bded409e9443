"""K1 (FrameAttention) timing + accuracy for both query conventions: plain q (scale in the kernel) and
q pre-multiplied by scale*log2(e) (the UNet's call: folded-max kernel at d = 40).
usage: python tools/k1_modes.py OUT.jsonl
Times the res-64 (d 40) and res-32 (d 80) launches of the edit (B=4, f=8) with HIP events and checks
a slice of each output against a float64 softmax(QK^T)V of the same bf16 inputs."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "video-p2p_amd"))
from vp2p import ops  # noqa: E402

out = sys.argv[1] if len(sys.argv) > 1 else "k1_modes.jsonl"
B, f, heads = 4, 8, 8
g = torch.Generator(device="cuda").manual_seed(0)
rows = []
for hw, C in ((4096, 320), (1024, 640)):
    d = C // heads
    c = ops.frame_query_scale(d)
    q = torch.randn(B * f, hw, C, device="cuda", dtype=torch.bfloat16, generator=g)
    k0 = torch.randn(B, hw, C, device="cuda", dtype=torch.bfloat16, generator=g)
    v0 = torch.randn(B, hw, C, device="cuda", dtype=torch.bfloat16, generator=g)
    for prescaled in (False, True):
        qq = (q.double() * c).bfloat16() if prescaled else q
        o = ops.frame_attention(qq, k0, v0, f, heads, q_prescaled=prescaled)
        bi, fi, nq = 1, 5, 512
        qs = qq[bi * f + fi, :nq].double().view(nq, heads, d).transpose(0, 1)
        ks = k0[bi].double().view(hw, heads, d).transpose(0, 1)
        vs = v0[bi].double().view(hw, heads, d).transpose(0, 1)
        ref = torch.softmax(qs @ ks.transpose(1, 2) * (1.0 / c if prescaled else 1.0) * d ** -0.5, -1) @ vs
        got = o[bi * f + fi, :nq].double().view(nq, heads, d).transpose(0, 1)
        err = ((got - ref).abs().max() / ref.abs().max()).item()
        for _ in range(3):
            ops.frame_attention(qq, k0, v0, f, heads, q_prescaled=prescaled)
        torch.cuda.synchronize()
        times = []
        for _ in range(5):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(10):
                ops.frame_attention(qq, k0, v0, f, heads, q_prescaled=prescaled)
            e.record()
            torch.cuda.synchronize()
            times.append(s.elapsed_time(e) / 10)
        times.sort()
        fl = 4.0 * B * f * hw * hw * C
        med = times[len(times) // 2]
        rows.append(dict(prescaled=prescaled, hw=hw, d=d, ms_median=round(med, 4), ms_min=round(times[0], 4),
                         tflops=round(fl / med / 1e9, 1), frac=round(fl / med / 1e9 / 2500, 4), rel_err=err))
with open(out, "a") as fh:
    for r in rows:
        print(json.dumps(r))
        fh.write(json.dumps(r) + "\n")
