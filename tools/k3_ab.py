"""Interleaved A/B of K3 (temporal attention + self-replace) between another build of the library
(A, --lib-a) and the in-tree one (B) at the B4 f8 edit shapes, inside and outside the self-replace
window; outputs must be bit-equal.  Kernel durations: run under rocprofv3 --kernel-trace."""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "video-p2p_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from vp2p import _lib, ops  # noqa: E402
from k2_ab import _Alt  # noqa: E402


def _err(o, q, k, v, f, heads, rep):
    """max |o - torch fp32 reference| / max |reference| of the temporal attention + self-replace."""
    Bf, n, C = q.shape
    B, d = Bf // f, C // heads
    t = lambda x: x.float().reshape(B, f, n, heads, d).permute(0, 2, 3, 1, 4)   # (B, n, h, f, d)  # noqa: E731
    s = torch.softmax(t(q) @ t(k).transpose(-1, -2) * d ** -0.5, -1)
    if rep:
        s[3] = s[2]                                   # cond half: edited prompt uses the source's maps
    ref = (s @ t(v)).permute(0, 3, 1, 2, 4).reshape(Bf, n, C)
    return float((o.float() - ref).abs().max() / ref.abs().max())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib-a", default=os.path.join(ROOT, "video-p2p_amd", "lib", "libvp2p_hip_prev.so"))
    ap.add_argument("--iters", type=int, default=10)
    args = ap.parse_args()
    lib_b = _lib.load()
    lib_a = _Alt(args.lib_a, lib_b)
    real = _lib.load
    B, f, heads = 4, 8, 8
    g = torch.Generator(device="cuda").manual_seed(0)
    flush = torch.empty(512 << 20, dtype=torch.uint8, device="cuda")   # > the 256 MB Infinity Cache
    for hw, C in ((4096, 320), (1024, 640), (256, 1280), (64, 1280)):
        qkv = torch.randn(B * f, hw, 3 * C, device="cuda", dtype=torch.bfloat16, generator=g)
        q, k, v = qkv[..., :C], qkv[..., C:2 * C], qkv[..., 2 * C:]
        for rep in (True, False):
            outs = {}
            for name, lib in (("A", lib_a), ("B", lib_b)):
                _lib.load = (lambda lib=lib: lib)
                for _ in range(args.iters):
                    flush.zero_()
                    o = ops.temporal_attention_p2p(q, k, v, f, heads, prompts=2, self_replace=rep)
                torch.cuda.synchronize()
                outs[name] = o
            _lib.load = real
            print(json.dumps({"hw": hw, "C": C, "self_replace": rep,
                              "bit_equal": bool(torch.equal(outs["A"], outs["B"])),
                              "max_abs_diff": float((outs["A"].float() - outs["B"].float()).abs().max()),
                              "ref_err_A": _err(outs["A"], q, k, v, f, heads, rep),
                              "ref_err_B": _err(outs["B"], q, k, v, f, heads, rep)}), flush=True)


if __name__ == "__main__":
    main()
