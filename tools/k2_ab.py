"""Interleaved A/B of the K2 cross-attention + P2P kernel: the in-tree library (B) against another
build of it (A, --lib-a; e.g. the previous kernel saved before a change).  Both run the edit the
bench runs (rabbit-jump AttentionRefine + Reweight, LocalBlend on at res-16) at the B4 f8 shapes;
outputs are compared (bit-equal O expected; LocalBlend sums within float reassociation).

Caveat: two loaded builds whose kernels have the SAME mangled name launch one code object (the
runtime resolves the kernel by name), so an A/B is only valid when the changed kernel's name or
signature differs between the builds; the bit-equality / reference checks catch a mix-up."""
import argparse
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "video-p2p_amd"))
sys.path.insert(0, ROOT)
import vp2p  # noqa: E402
from vp2p import _lib, ops  # noqa: E402
from vp2p.tokenizer import SyntheticCLIPTokenizer  # noqa: E402


class _Alt:
    """Another build of the library, exposing the in-tree library's ctypes signatures."""

    def __init__(self, path, ref):
        self._lib, self._ref = ctypes.CDLL(path), ref

    def __getattr__(self, name):
        fn = getattr(self._lib, name)
        src = getattr(self._ref, name)
        fn.argtypes, fn.restype = src.argtypes, src.restype
        return fn


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib-a", default=os.path.join(ROOT, "video-p2p_amd", "lib", "libvp2p_hip_k2old.so"))
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--frames", type=int, default=8)
    args = ap.parse_args()
    lib_b = _lib.load()
    lib_a = _Alt(args.lib_a, lib_b)
    real_load = _lib.load
    bench = __import__("bench")
    prompts, swap, blend, eq, cross, self_ = bench.RABBIT
    ctrl = vp2p.make_controller(prompts, swap, {"default_": cross}, self_, blend, eq,
                                tokenizer=SyntheticCLIPTokenizer(), num_steps=50)
    plan = ctrl.plan("cuda")
    B, f, heads = 4, args.frames, 8
    dt = torch.bfloat16
    g = torch.Generator(device="cuda").manual_seed(0)
    out = []
    for hw, C in ((4096, 320), (1024, 640), (256, 1280), (64, 1280)):
        q = torch.randn(B * f, hw, C, device="cuda", dtype=dt, generator=g)
        k = torch.randn(B, 77, C, device="cuda", dtype=dt, generator=g)
        v = torch.randn(B, 77, C, device="cuda", dtype=dt, generator=g)
        use_lb = hw == 256
        res = {}
        outs = {}
        for name, lib in (("A", lib_a), ("B", lib_b)):
            _lib.load = (lambda lib=lib: lib)
            lb = torch.zeros(2, f, hw, device="cuda") if use_lb else None
            o = ops.cross_attention_p2p(q, k, v, f, heads, plan=plan, step=3, lb_acc=lb)
            outs[name] = (o.clone(), None if lb is None else lb.clone())
        _lib.load = real_load
        same_o = bool(torch.equal(outs["A"][0], outs["B"][0]))
        lb_err = None if not use_lb else float((outs["A"][1] - outs["B"][1]).abs().max() /
                                               outs["A"][1].abs().max())
        times = {"A": [], "B": []}
        for _ in range(args.rounds):
            for name, lib in (("A", lib_a), ("B", lib_b)):
                _lib.load = (lambda lib=lib: lib)
                lb = torch.zeros(2, f, hw, device="cuda") if use_lb else None
                for _ in range(3):
                    ops.cross_attention_p2p(q, k, v, f, heads, plan=plan, step=3, lb_acc=lb)
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                s.record()
                for _ in range(args.iters):
                    ops.cross_attention_p2p(q, k, v, f, heads, plan=plan, step=3, lb_acc=lb)
                e.record()
                torch.cuda.synchronize()
                times[name].append(s.elapsed_time(e) / args.iters * 1e3)
        _lib.load = real_load
        byt = 2.0 * B * f * hw * C * 2
        for name in ("A", "B"):
            t = sorted(times[name])[len(times[name]) // 2]
            res[name] = {"us": round(t, 2), "GBps": round(byt / t / 1e3, 1)}
        row = {"hw": hw, "C": C, "lb": use_lb, "A": res["A"], "B": res["B"], "O_bit_equal": same_o,
               "lb_rel_err": lb_err}
        print(json.dumps(row), flush=True)
        out.append(row)


if __name__ == "__main__":
    main()
