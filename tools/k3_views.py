"""K3 (attn_temp) at the UNet's layout: q, k, v as column views of one fused (B*f*N, 3C) qkv GEMM
output (attention.py:262-268 on the fused projection), HIP-event median; checksum for A/B.
usage: python tools/k3_views.py OUT.jsonl   (library from VP2P_LIB)"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "video-p2p_amd"))
from vp2p import ops  # noqa: E402

lib = os.path.basename(os.environ.get("VP2P_LIB", "libvp2p_hip.so"))
rows = []
B, f, heads = 4, 8, 8
g = torch.Generator(device="cuda").manual_seed(0)
for hw, C in ((4096, 320), (1024, 640), (256, 1280), (64, 1280)):
    qkv = torch.randn(B * f, hw, 3 * C, device="cuda", generator=g).bfloat16()
    q, k, v = qkv[..., :C], qkv[..., C:2 * C], qkv[..., 2 * C:]
    o = ops.temporal_attention_p2p(q, k, v, f, heads, prompts=2, self_replace=True)
    for _ in range(3):
        ops.temporal_attention_p2p(q, k, v, f, heads, prompts=2, self_replace=True)
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(20):
            ops.temporal_attention_p2p(q, k, v, f, heads, prompts=2, self_replace=True)
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e) / 20)
    t = sorted(ts)[2]
    byt = 4.0 * B * f * hw * C * 2
    r = dict(lib=lib, hw=hw, d=C // heads, us=round(t * 1e3, 2), gbs=round(byt / t / 1e6, 1),
             checksum=o.float().abs().sum().item())
    print(json.dumps(r), flush=True)
    rows.append(r)
with open(sys.argv[1], "a") as fh:
    for r in rows:
        fh.write(json.dumps(r) + "\n")
