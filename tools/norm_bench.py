"""Time K7 (GroupNorm+add+SiLU), K8 (LayerNorm), K9 (GEGLU) against the torch ops they replace, at
the res-64 edit shapes (B=4, f=8, 64x64, C=320, bf16).  Prints one JSON line per op with the
algorithmic bytes and the achieved HBM bandwidth."""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "video-p2p_amd"))
from vp2p import ops  # noqa: E402


def timeit(fn, n=50):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3  # us


def main():
    dt = torch.bfloat16
    B, f, C, H = 4, 8, 320, 64
    x = torch.randn(B * f, C, H, H, device="cuda", dtype=dt).to(memory_format=torch.channels_last)
    t = torch.randn(B * f, C, device="cuda", dtype=dt)
    gn = torch.nn.GroupNorm(32, C).cuda().to(dt)
    res = []
    nb = x.numel() * 2
    with torch.no_grad():
        k = timeit(lambda: ops.group_norm(x, 32, gn.weight, gn.bias, 1e-5, f, silu=True, add=t))

    def torch_gn():
        xx = x + t[:, :, None, None]
        x5 = xx.reshape(B, f, C, H, H).permute(0, 2, 1, 3, 4)
        return F.silu(F.group_norm(x5, 32, gn.weight, gn.bias, 1e-5))
    with torch.no_grad():
        tt = timeit(torch_gn)
    res.append({"op": "K7 group_norm+add+silu", "shape": [B * f, C, H, H], "us": round(k, 2),
                "torch_us": round(tt, 2), "alg_bytes": 2 * nb, "GB/s": round(2 * nb / k / 1e3, 1)})
    rows = B * f * H * H
    xl = torch.randn(rows, C, device="cuda", dtype=dt)
    ln = torch.nn.LayerNorm(C).cuda().to(dt)
    with torch.no_grad():
        k = timeit(lambda: ops.layer_norm(xl, ln.weight, ln.bias, 1e-5))
        tt = timeit(lambda: ln(xl))
    res.append({"op": "K8 layer_norm", "shape": [rows, C], "us": round(k, 2), "torch_us": round(tt, 2),
                "alg_bytes": 2 * xl.numel() * 2, "GB/s": round(4 * xl.numel() / k / 1e3, 1)})
    hg = torch.randn(rows, 8 * C, device="cuda", dtype=dt)
    with torch.no_grad():
        k = timeit(lambda: ops.geglu(hg))

        def tg():
            a, g = hg.chunk(2, dim=-1)
            return a * F.gelu(g)
        tt = timeit(tg)
    byt = hg.numel() * 2 + hg.numel()
    res.append({"op": "K9 geglu", "shape": [rows, 8 * C], "us": round(k, 2), "torch_us": round(tt, 2),
                "alg_bytes": byt, "GB/s": round(byt / k / 1e3, 1)})
    for r in res:
        print(json.dumps(r))


if __name__ == "__main__":
    main()
