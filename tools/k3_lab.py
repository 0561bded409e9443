"""K3 A/B over lab builds: each library in argv runs in its own child process (VP2P_LIB) and times
the temporal attention + self-replace launches of the edit (B=4 f=8, the qkv GEMM's interleaved
layout, in and out of the self-replace window) with HIP events, plus an output checksum (builds of
the same arithmetic must agree bit for bit) and the error against a torch fp32 reference.
usage: python tools/k3_lab.py OUT.jsonl lib1.so [lib2.so ...]   (rounds alternate the libraries)"""
import json
import os
import subprocess
import sys

CHILD = r'''
import json, os, sys, torch
sys.path.insert(0, os.path.join(os.environ["VP2P_ROOT"], "video-p2p_amd"))
from vp2p import ops
B, f, heads = 4, 8, 8
g = torch.Generator(device="cuda").manual_seed(0)
rows = []
for hw, C in ((4096, 320), (1024, 640), (256, 1280), (64, 1280)):
    d = C // heads
    qkv = torch.randn(B * f, hw, 3 * C, device="cuda", dtype=torch.bfloat16, generator=g)
    q, k, v = qkv[..., :C], qkv[..., C:2 * C], qkv[..., 2 * C:]
    for rep in (True, False):
        o = ops.temporal_attention_p2p(q, k, v, f, heads, prompts=2, self_replace=rep)
        t = lambda x: x.float().reshape(B, f, hw, heads, d).permute(0, 2, 3, 1, 4)
        s = torch.softmax(t(q) @ t(k).transpose(-1, -2) * d ** -0.5, -1)
        if rep:
            s[3] = s[2]
        ref = (s @ t(v)).permute(0, 3, 1, 2, 4).reshape(B * f, hw, C)
        err = float((o.float() - ref).abs().max() / ref.abs().max())
        for _ in range(3):
            ops.temporal_attention_p2p(q, k, v, f, heads, prompts=2, self_replace=rep)
        torch.cuda.synchronize()
        times = []
        for _ in range(7):
            s0, e0 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s0.record()
            for _ in range(10):
                ops.temporal_attention_p2p(q, k, v, f, heads, prompts=2, self_replace=rep)
            e0.record()
            torch.cuda.synchronize()
            times.append(s0.elapsed_time(e0) / 10)
        times.sort()
        med = times[len(times) // 2]
        # algorithmic bytes: q, k read for the prompts whose scores are computed, v read, o written
        nqk = 3 if rep else 4
        byt = (nqk * 2 + 4 + 4) * f * hw * C * 2
        rows.append(dict(lib=os.path.basename(os.environ["VP2P_LIB"]), hw=hw, d=d, self_replace=rep,
                         ms_median=round(med, 4), ms_min=round(times[0], 4), tbs=round(byt / med / 1e9, 3),
                         frac=round(byt / med / 1e9 / 8.0, 4), rel_err=err, abs_sum=o.float().abs().sum().item()))
print("ROWS" + json.dumps(rows))
'''

out, libs = sys.argv[1], sys.argv[2:]
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
with open(out, "a") as fh:
    for rnd in range(2):
        for lib in libs:
            env = dict(os.environ, VP2P_LIB=os.path.abspath(lib), VP2P_ROOT=root)
            r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
            if r.returncode != 0:
                print(f"{lib}: rc {r.returncode}\n{r.stderr[-2000:]}", flush=True)
                sys.exit(r.returncode)
            for row in json.loads(r.stdout.split("ROWS", 1)[1]):
                row["round"] = rnd
                print(json.dumps(row), flush=True)
                fh.write(json.dumps(row) + "\n")
