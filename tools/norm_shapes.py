"""K7 GroupNorm (+temb add, SiLU) and K8 LayerNorm (+ residual add) at every UNet3D shape of the B4
f8 512^2 edit, N launches each, for rocprofv3 --kernel-trace (per-launch durations by shape).
Prints the algorithmic bytes per launch of each op/shape in launch order.  A/B caveat as in
tools/k2_ab.py: kernels with the same mangled name in both builds run one code object."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "video-p2p_amd"))
from vp2p import ops  # noqa: E402


_REAL = None


def _use(lib):
    """Route vp2p.ops through `lib` (None: the in-tree library)."""
    global _REAL
    from vp2p import _lib
    if _REAL is None:
        _REAL = _lib.load
    _lib.load = _REAL if lib is None else (lambda path=None, lib=lib: lib)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    libs = [None]
    if len(sys.argv) > 2:          # A/B: another build first, then the in-tree library, per shape
        from vp2p import _lib
        other = _lib.load(sys.argv[2])
        real = _lib.load()
        libs = [other, real]
    dt = torch.bfloat16
    B, f = 4, 8
    out = []
    for C, H in ((320, 64), (640, 32), (1280, 16), (1280, 8), (640, 64), (960, 64), (960, 32), (1920, 32),
                 (1920, 16), (2560, 16), (2560, 8)):
        x = torch.randn(B * f, C, H, H, device="cuda", dtype=dt).to(memory_format=torch.channels_last)
        t = torch.randn(B * f, C, device="cuda", dtype=dt)
        w = torch.ones(C, device="cuda", dtype=dt)
        bs = torch.zeros(C, device="cuda", dtype=dt)
        for lib in libs:
            _use(lib)
            with torch.no_grad():
                for _ in range(n):
                    ops.group_norm(x, 32, w, bs, 1e-5, f, silu=True, add=t)
                for _ in range(n):
                    ops.group_norm(x, 32, w, bs, 1e-6, f, silu=False)
        out.append({"op": "gn", "C": C, "H": H, "x_bytes": x.numel() * 2})
    for C, H in ((320, 64), (640, 32), (1280, 16), (1280, 8)):
        xl = torch.randn(B * f * H * H, C, device="cuda", dtype=dt)
        r = torch.randn_like(xl)
        w = torch.ones(C, device="cuda", dtype=dt)
        bs = torch.zeros(C, device="cuda", dtype=dt)
        for lib in libs:
            _use(lib)
            with torch.no_grad():
                for _ in range(n):
                    ops.layer_norm(xl, w, bs, 1e-5)
        out.append({"op": "ln", "C": C, "H": H, "x_bytes": xl.numel() * 2})
    torch.cuda.synchronize()
    for o in out:
        print(json.dumps(o))


if __name__ == "__main__":
    main()
