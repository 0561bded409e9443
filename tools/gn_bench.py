"""K7 GroupNorm at the UNet's shapes (B=4 x f=8, 512^2): stats kernel, the per-block-merge apply
(vp2p_group_norm_apply) and the finalize + apply_stats pair; HIP-event medians and the max
difference between the two applies.  usage: python tools/gn_bench.py OUT.jsonl"""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "video-p2p_amd"))
from vp2p import _lib, ops  # noqa: E402


def med(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(n):
            fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e) / n * 1e3)
    return sorted(ts)[2]


lib = _lib.load()
B, f, G = 4, 8, 32
rows = []
for C, H in ((320, 64), (640, 64), (960, 64), (640, 32), (1280, 32), (1920, 32), (1280, 16), (2560, 16), (1280, 8)):
    for silu in (False, True):
        x = torch.randn(B * f, C, H, H, device="cuda").bfloat16().to(memory_format=torch.channels_last)
        w = torch.randn(C, device="cuda").bfloat16()
        bb = torch.randn(C, device="cuda").bfloat16()
        add = torch.randn(B * f, C, device="cuda").bfloat16() if silu else None
        y1, y2 = torch.empty_like(x), torch.empty_like(x)
        a = ops._gn_args(x, G, w, bb, 1e-5, f, silu, add, y1)
        parts = lib.vp2p_group_norm_parts(ctypes.byref(a))
        partials = torch.empty(B * parts * G * 3, device="cuda")
        st = torch.empty(B * G * 2, device="cuda")
        a.partials = partials.data_ptr()
        s = ops._stream()
        t_stats = med(lambda: lib.vp2p_group_norm_stats(ctypes.byref(a), s))
        t_old = med(lambda: lib.vp2p_group_norm_apply(ctypes.byref(a), ctypes.c_void_p(partials.data_ptr()), 1, s))
        a2 = ops._gn_args(x, G, w, bb, 1e-5, f, silu, add, y2)
        a2.partials = partials.data_ptr()
        t_fin = med(lambda: lib.vp2p_group_norm_finalize(ctypes.byref(a2), ctypes.c_void_p(partials.data_ptr()), 1,
                                                          ctypes.c_void_p(st.data_ptr()), s))
        t_app = med(lambda: lib.vp2p_group_norm_apply_stats(ctypes.byref(a2), ctypes.c_void_p(st.data_ptr()), s))
        torch.cuda.synchronize()
        mb = x.numel() * 2 / 1e6
        r = dict(C=C, H=H, silu=silu, MB=round(mb, 1), stats_us=round(t_stats, 1), apply_old_us=round(t_old, 1),
                 finalize_us=round(t_fin, 1), apply_stats_us=round(t_app, 1),
                 apply_GBps=round(2 * mb * 1e3 / t_app, 0),
                 maxdiff=(y1.float() - y2.float()).abs().max().item(), sum=y2.double().abs().sum().item(),
                 stats_sum=partials.double().abs().sum().item())
        print(json.dumps(r), flush=True)
        rows.append(r)
with open(sys.argv[1], "a") as fh:
    for r in rows:
        fh.write(json.dumps(r) + "\n")
