"""K3 at the edit's res-64 shape (B4 f8, 4096 tokens, C 320, q|k|v slices of one projection): the
persistent stream (K3s, ring depth 2 / 3 / 4) against the short kernel (VP2P_K3_STREAM=0), self-replace on and off, plus
the cond-only half; per-launch time by HIP events on the launch stream, median over reps, with the
Infinity Cache flushed before each launch (as in the edit, where the operands come from HBM).
    python tools/k3_stream_ab.py OUT.jsonl"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "video-p2p_amd"))
from vp2p import ops  # noqa: E402


# VP2P_K3_STREAM: the short kernel, stream ring depths 2 / 3 / 4 (K3AB_MODES / K3AB_SHAPES narrow it)
MODES = tuple(os.environ.get("K3AB_MODES", "0,2,3,4").split(","))
SHAPES = ((4096, 320), (1024, 640))[:int(os.environ.get("K3AB_SHAPES", "2"))]
PRODUCER = os.environ.get("K3AB_PRODUCER", "1") == "1"   # 0: flush the Infinity Cache before each launch


def main():
    out_path = sys.argv[1] if len(sys.argv) > 1 else "k3_stream_ab.jsonl"
    f, heads, reps = 8, 8, 30
    g = torch.Generator(device="cuda").manual_seed(0)
    flush = torch.empty(512 << 20, dtype=torch.uint8, device="cuda")
    lines = []
    for hw, C in SHAPES:
        for B, kw, name in ((4, dict(prompts=2, self_replace=True), "replace"),
                            (4, dict(prompts=2, self_replace=False), "edit"),
                            (2, dict(prompts=2, self_replace=True, cond_only=True), "cond_only"),
                            (2, {}, "plain2")):
            qkv = torch.randn(B * f, hw, 3 * C, device="cuda", dtype=torch.bfloat16, generator=g)
            q, k, v = qkv[..., :C], qkv[..., C:2 * C], qkv[..., 2 * C:]
            zero = torch.zeros((), device="cuda", dtype=torch.bfloat16)
            res = {}
            outs = {}
            for mode in MODES + MODES:
                os.environ["VP2P_K3_STREAM"] = mode
                ts = []
                for _ in range(reps):
                    if PRODUCER:
                        qkv.add_(zero)         # the projection that writes q|k|v right before K3 (as in the edit)
                    else:
                        flush.zero_()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    o = ops.temporal_attention_p2p(q, k, v, f, heads, **kw)
                    e1.record()
                    torch.cuda.synchronize()
                    ts.append(e0.elapsed_time(e1) * 1e3)
                ts.sort()
                res.setdefault(mode, []).append(ts[len(ts) // 2])
                outs[mode] = o
            # bytes as the bench counts them (q, k, v in + o out for every row, 8 C B per row)
            rows = B * f * hw
            d = {"hw": hw, "C": C, "case": name, "bytes_bench_convention": rows * C * 2 * 4}
            for m in MODES:
                d[f"us_{m}"] = min(res[m])
                d[f"TBps_{m}"] = d["bytes_bench_convention"] / d[f"us_{m}"] / 1e6
                d[f"bit_equal_{m}"] = bool(torch.equal(outs[MODES[0]], outs[m]))
            d["lib"] = os.path.basename(os.environ.get("VP2P_LIB", "libvp2p_hip.so"))
            print(json.dumps(d), flush=True)
            lines.append(d)
    os.environ.pop("VP2P_K3_STREAM", None)
    with open(out_path, "w") as fh:
        for d in lines:
            fh.write(json.dumps(d) + "\n")


if __name__ == "__main__":
    main()
