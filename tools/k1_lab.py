"""K1 A/B over lab builds: each library in argv runs in its own child process (VP2P_LIB) and times
the res-64 (d 40, pre-scaled q: the UNet's call), res-32 (d 80), res-16 and res-8 (d 160) FrameAttention launches of the
edit (B=4, f=8) with HIP events, checking a slice against a float64 softmax(QK^T)V.
usage: python tools/k1_lab.py OUT.jsonl lib1.so [lib2.so ...]   (rounds alternate the libraries)"""
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
    c = ops.frame_query_scale(d)
    q = torch.randn(B * f, hw, C, device="cuda", dtype=torch.bfloat16, generator=g)
    k0 = torch.randn(B, hw, C, device="cuda", dtype=torch.bfloat16, generator=g)
    v0 = torch.randn(B, hw, C, device="cuda", dtype=torch.bfloat16, generator=g)
    qq = (q.double() * c).bfloat16()
    o = ops.frame_attention(qq, k0, v0, f, heads, q_prescaled=True)
    bi, fi, nq = 1, 5, min(512, hw)
    qs = qq[bi * f + fi, :nq].double().view(nq, heads, d).transpose(0, 1)
    ks = k0[bi].double().view(hw, heads, d).transpose(0, 1)
    vs = v0[bi].double().view(hw, heads, d).transpose(0, 1)
    ref = torch.softmax(qs @ ks.transpose(1, 2) / c * d ** -0.5, -1) @ vs
    got = o[bi * f + fi, :nq].double().view(nq, heads, d).transpose(0, 1)
    err = ((got - ref).abs().max() / ref.abs().max()).item()
    full = o.float().abs().sum().item()
    for _ in range(3):
        ops.frame_attention(qq, k0, v0, f, heads, q_prescaled=True)
    torch.cuda.synchronize()
    times = []
    for _ in range(7):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(10):
            ops.frame_attention(qq, k0, v0, f, heads, q_prescaled=True)
        e.record()
        torch.cuda.synchronize()
        times.append(s.elapsed_time(e) / 10)
    times.sort()
    fl = 4.0 * B * f * hw * hw * C
    med = times[len(times) // 2]
    rows.append(dict(lib=os.path.basename(os.environ["VP2P_LIB"]), hw=hw, d=d, ms_median=round(med, 4),
                     ms_min=round(times[0], 4), tflops=round(fl / med / 1e9, 1),
                     frac=round(fl / med / 1e9 / 2500, 4), rel_err=err, abs_sum=full))
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
            rows = json.loads(r.stdout.split("ROWS", 1)[1])
            for row in rows:
                row["round"] = rnd
                print(json.dumps(row), flush=True)
                fh.write(json.dumps(row) + "\n")
