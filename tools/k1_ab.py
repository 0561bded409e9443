"""Interleaved A/B of K1 schedule variants in one process (VP2P_K1_VARIANT read per launch)."""
import os
import sys
import statistics
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "video-p2p_amd"))
from vp2p import ops  # noqa: E402

variants = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "2,4").split(",")]
B, f, heads = 4, 8, 8
for hw, C in ((4096, 320), (1024, 640)):
    q = torch.randn(B * f, hw, C, device="cuda", dtype=torch.bfloat16)
    k0 = torch.randn(B, hw, C, device="cuda", dtype=torch.bfloat16)
    v0 = torch.randn(B, hw, C, device="cuda", dtype=torch.bfloat16)
    ref = None
    res = {v: [] for v in variants}
    for rnd in range(8):
        for v in variants:
            os.environ["VP2P_K1_VARIANT"] = str(v)
            out = ops.frame_attention(q, k0, v0, f, heads)
            if ref is None:
                ref = out.float()
            elif rnd == 0:
                assert (out.float() - ref).abs().max().item() < 2e-2, v
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(10):
                ops.frame_attention(q, k0, v0, f, heads)
            e.record()
            torch.cuda.synchronize()
            res[v].append(s.elapsed_time(e) / 10)
    fl = 4.0 * B * f * hw * hw * C
    for v in variants:
        med = statistics.median(res[v])
        print(f"hw={hw} d={C // heads} var={v} median {med:.4f} ms min {min(res[v]):.4f} -> {fl / med / 1e9:.1f} TF/s")
