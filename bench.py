#!/usr/bin/env python
"""Benchmark: edited frames/s of a 50-step DDIM Video-P2P edit at 512^2 (BASELINE.json metric).

One "step" = one complete edit of one clip: 50 denoising steps of the UNet3D at batch 4
(2 prompts x CFG) with the P2P controller (AttentionRefine + LocalBlend + AttentionReweight of
configs/rabbit-jump-p2p.yaml), fast mode, DDIM eta = 0 -- configs[1] of BASELINE.json
("rabbit-jump-p2p 8f 512^2 on 1xMI355X bf16").  Synthetic data: random-init SD-1.5-geometry
UNet3D (seed 0, N(0, 0.02), attn_temp.to_out non-zero), random text embeddings standing in for
CLIP (seed 1; CLIP and VAE are excluded from the metric), x_T ~ N(0, 1) (seed 2 + rank).

Multi-GPU (torchrun): every rank edits its own clip, no data-path collective (scaling "weak");
value = clips * frames / max-over-ranks wall time.

The JSON line also carries the live roofline of K1 (frame attention, the dominant, MFMA-bound
kernel: its res-64 launch timed with HIP events on the launch stream during the timed region) and
a CPU baseline (rank 0, N = 1): the oracle's fp32 CPU path on a bounded per-block sample,
extrapolated to the same edit.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "video-p2p_amd"))

import torch  # noqa: E402

PEAK_BF16_TFLOPS = 2500.0      # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
PEAK_F32_TFLOPS = 157.3
RABBIT = (["a rabbit is jumping on the grass", "a origami rabbit is jumping on the grass"],
          False, (("rabbit",), ("rabbit",)), {"words": ["origami"], "values": [2]}, 0.2, 0.5)
# The other reference edits (configs/*-p2p.yaml; cross 0.2 / self 0.5 are run_videop2p.py's defaults).
EDITS = {
    "rabbit": ("rabbit-jump-p2p", "AttentionRefine+LocalBlend+Reweight", RABBIT),
    "penguin": ("penguin-run-p2p", "AttentionRefine+LocalBlend+Reweight",
                (["a penguin is running on the ice", "a crochet penguin is running on the ice"],
                 False, (("penguin",), ("penguin",)), {"words": ["crochet"], "values": [4]}, 0.2, 0.5)),
    "car": ("car-drive-p2p", "AttentionReplace+LocalBlend+Reweight",
            (["a car is driving on the road", "a car is driving on the railway"],
             True, (("road",), ("railway",)), {"words": ["railway"], "values": [2]}, 0.2, 0.5)),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2, help="timed edits (each = 50 DDIM steps)")
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--frames", type=int, default=8)
    ap.add_argument("--edit", default="rabbit", choices=sorted(EDITS),
                    help="which reference edit (configs/<name>-p2p.yaml): rabbit = configs[1] (default), "
                         "penguin --frames 24 = configs[2], car = the word-swap AttentionReplace path")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--ddim-steps", type=int, default=50)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-k1-events", action="store_true")
    ap.add_argument("--mode", default="edit", choices=["edit", "nulltext", "k1long"],
                    help="edit: the P2P edit (BASELINE metric, configs[1]); nulltext: official-mode inversion "
                         "(DDIM inversion + null-text optimisation, configs[3]), one step = one inversion; "
                         "k1long: configs[4], the FrameAttention of one UNet forward over a --long-frames clip "
                         "at 768^2, frames sharded over the ranks with the RCCL frame-0 K/V broadcast")
    ap.add_argument("--long-frames", type=int, default=128, help="k1long: frames of the clip")
    ap.add_argument("--conv-find", type=int, default=0,
                    help="1: run MIOpen's solver search per new conv shape (torch.backends.cudnn.benchmark; slow "
                         "warmup); 0 (default): immediate mode, which takes the tuned solvers recorded in the "
                         "in-tree database miopen_db/ (tools/miopen_tune.py)")
    ap.add_argument("--tuned", type=int, default=1,
                    help="1 (default): in-tree tuned MIOpen database (vp2p.tuning); 0: library heuristics")
    ap.add_argument("--inner-steps", type=int, default=10, help="null-text Adam iterations per DDIM step")
    ap.add_argument("--shard", default="clips", choices=["clips", "frames"],
                    help="clips: every rank edits its own clip (weak scaling, no collective); "
                         "frames: one clip's frames split over the ranks (strong scaling, RCCL)")
    return ap.parse_args()


class K1Timer:
    """Brackets every res-64 FrameAttention launch with HIP events on the launch stream."""

    def __init__(self, ops, tokens=4096):
        self.ops, self.tokens, self.orig = ops, tokens, ops.frame_attention
        self.events, self.active = [], False

    def __enter__(self):
        orig = self.orig

        def wrapped(q, *a, **k):
            if not self.active or q.shape[1] != self.tokens:
                return orig(q, *a, **k)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            out = orig(q, *a, **k)
            e.record()
            self.events.append((s, e, tuple(q.shape)))
            return out

        self.ops.frame_attention = wrapped
        import vp2p.attention as att
        att.ops.frame_attention = wrapped
        return self

    def __exit__(self, *exc):
        self.ops.frame_attention = self.orig

    def summary(self, frames, peak):
        if not self.events:
            return None
        ms = [s.elapsed_time(e) for s, e, _ in self.events]
        Bf, N, C = self.events[0][2]
        flops = 4.0 * Bf * N * N * C           # QK^T + PV, frame-0 K/V: 4 * B*f * HW^2 * C
        avg_s = sum(ms) / len(ms) / 1e3
        achieved = flops / avg_s / 1e12
        esz = 2 if peak == PEAK_BF16_TFLOPS else 4
        alg_bytes = esz * (2 * Bf * N * C + 2 * (Bf // frames) * N * C)   # Q in + O out + frame-0 K, V
        traffic, src = _pmc_traffic()
        return {"bound": "mfma", "achieved": round(achieved, 1), "peak": peak, "unit": "TFLOP/s",
                "frac": round(achieved / peak, 4), "traffic": traffic, "traffic_unit": "bytes/launch",
                "traffic_source": src, "algorithmic_bytes": alg_bytes,
                "kernel": "vp2p::frame_attn_kernel_x2f<40,256> (res-64 FrameAttention, bf16)",
                "launches": len(ms), "avg_ms": round(sum(ms) / len(ms), 4),
                "flops_per_launch": flops}


TRAFFIC_FILE = os.path.join(ROOT, "profiles", "k1_pmc_traffic.json")


def _pmc_traffic():
    """HBM bytes per K1 launch from the committed rocprofv3 --pmc passes (FETCH_SIZE x2 per the gfx950
    correction, + WRITE_SIZE; tools/pmc_traffic.py) on the same kernel and shape, or None."""
    try:
        with open(TRAFFIC_FILE) as fh:
            d = json.load(fh)
        return d["bytes_per_launch"], os.path.relpath(TRAFFIC_FILE, ROOT) + " (" + d["how"] + ")"
    except (OSError, KeyError, ValueError):
        return None, None


def cpu_baseline(frames, ddim_steps, threads):
    """Oracle fp32 CPU path on a bounded sample: one transformer block and one resnet block per
    resolution level of the B=4 edit UNet, extrapolated by the block counts of one forward and x50."""
    import numpy as np
    from oracle import p2p_oracle as O
    from oracle import unet_ref
    from vp2p.tokenizer import SyntheticCLIPTokenizer
    from vp2p.unet3d import UNet3DConditionModel, init_random_
    torch.set_num_threads(threads)
    prompts, swap, blend, eq, cross, self_ = RABBIT
    tok = SyntheticCLIPTokenizer()
    ctrl = O.EditController(prompts, swap, {"default_": cross}, self_, tok, blend_words=blend, eq_params=eq)
    sd = {k: v for k, v in init_random_(UNet3DConditionModel(), seed=0).state_dict().items()}
    g = torch.Generator().manual_seed(3)
    B = 4
    ctx = torch.randn(B, 77, 768, generator=g)
    emb = torch.randn(B, 1280, generator=g)
    # (prefix of a transformer, prefix of a resnet, channels, latent size, transformers, resnets per forward)
    levels = [("down_blocks.0.attentions.0.", "down_blocks.0.resnets.1.", 320, 64, 5, 5),
              ("down_blocks.1.attentions.0.", "down_blocks.1.resnets.1.", 640, 32, 5, 5),
              ("down_blocks.2.attentions.0.", "down_blocks.2.resnets.1.", 1280, 16, 5, 5),
              ("mid_block.attentions.0.", "mid_block.resnets.0.", 1280, 8, 1, 7)]
    t_fwd, t_sample = 0.0, 0.0
    for tp, rp, C, hw, n_t, n_r in levels:
        x = torch.randn(B, C, frames, hw, hw, generator=g) * 0.5
        t0 = time.perf_counter()
        with torch.no_grad():
            unet_ref.transformer(sd, tp, x, ctx, ctrl, "down")
        t1 = time.perf_counter()
        with torch.no_grad():
            unet_ref.resnet(sd, rp, x, emb)
        t2 = time.perf_counter()
        t_fwd += n_t * (t1 - t0) + n_r * (t2 - t1)
        t_sample += t2 - t0
    t_edit = t_fwd * ddim_steps
    return {"value": round(frames / t_edit, 6), "unit": "edited frames/s", "cores": threads, "kind": "port",
            "sample": (f"oracle/unet_ref.py fp32 on host CPU: 1 transformer block + 1 resnet block per level "
                       f"(B=4, f={frames}, 512^2) timed once ({t_sample:.1f} s), extrapolated by block counts to "
                       f"one UNet forward ({t_fwd:.1f} s) x {ddim_steps} steps; excludes up/downsample convs"),
            "cpu_model": _cpu_model()}


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def k1long_main(args, world, rank, dev):
    """configs[4] of BASELINE.json: sparse-causal (first-frame K/V) attention of a 128-frame 768^2
    clip, sharded by frames over the ranks.  One step = every attn1 call of one UNet forward at
    UNet batch 4 (5 blocks at 96^2 tokens / C 320, 5 at 48^2 / 640, 5 at 24^2 / 1280, 1 at 12^2 / 1280):
    per call rank 0 (owner of frame 0) broadcasts the frame-0 K/V (B, HW, 2C) over RCCL, then every
    rank runs K1 on its f/G frames.  Synthetic bf16 activations; the projections are not timed."""
    import torch.distributed as dist
    from vp2p import ops
    B, heads, f = 4, 8, args.long_frames
    if f % world:
        raise SystemExit(f"--long-frames {f} does not split over {world} ranks")
    fl = f // world
    levels = [(96 * 96, 320, 5), (48 * 48, 640, 5), (24 * 24, 1280, 5), (12 * 12, 1280, 1)]
    g = torch.Generator(device=dev).manual_seed(3 + rank)
    bufs = []
    for hw, C, n in levels:
        q = torch.randn(B * fl, hw, C, device=dev, dtype=torch.bfloat16, generator=g)
        kv = torch.randn(B, hw, 2 * C, device=dev, dtype=torch.bfloat16, generator=g)
        bufs.append((q, kv, torch.empty_like(q), C, n))

    def step():
        for q, kv, out, C, n in bufs:
            for _ in range(n):
                if world > 1:
                    dist.broadcast(kv, src=0)
                ops.frame_attention(q, kv[..., :C], kv[..., C:], fl, heads, out=out)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    flops = sum(4.0 * B * f * hw * hw * C * n for hw, C, n in levels)
    result = {
        "metric": "sparse-causal attention TFLOP/s, 768^2 x 128-frame clip (K1 + RCCL frame-0 K/V broadcast)",
        "value": round(flops * args.steps / elapsed / 1e12, 1), "unit": "TFLOP/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 2), "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "bf16", "data": "synthetic (random bf16 q / frame-0 k,v)",
        "config": {"workload": f"attn1 of one UNet forward, {f} frames 768^2, UNet batch {B}, frame-sharded x{world}",
                   "frames": f, "resolution": 768, "unet_batch": B, "parallelism": f"frame-sharded x{world} (RCCL)"},
        "frames_per_s": round(f * args.steps / elapsed, 2),
        "roofline": {"bound": "mfma", "achieved": round(flops / world * args.steps / elapsed / 1e12, 1),
                     "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                     "frac": round(flops / world * args.steps / elapsed / 1e12 / PEAK_BF16_TFLOPS, 4),
                     "note": "per-GPU K1 algorithmic FLOP rate including the broadcast time"},
    }
    if rank == 0:
        print(json.dumps(result), flush=True)


def nulltext_main(args, world, rank, dev):
    """configs[3] of BASELINE.json: NullInversion.invert (run_videop2p.py:614-624) of an 8-frame 512^2
    clip: 50 DDIM-inversion steps, then per step one conditional forward, up to --inner-steps
    forward+backward Adam iterations (random weights never reach the early-stop epsilon, so always
    the maximum, the reference's worst case) and one guided step (B=2).  Clip-parallel over ranks."""
    from vp2p.pipeline import NullInversion, VideoP2PPipeline
    from vp2p.unet3d import UNet3DConditionModel, init_random_
    dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    unet = init_random_(UNet3DConditionModel(), seed=0).to(dev, dtype).to(memory_format=torch.channels_last)
    unet.eval()
    g = torch.Generator().manual_seed(1)
    ctx = torch.randn(2, 77, 768, generator=g).to(dev)
    x0 = torch.randn(1, 4, args.frames, 64, 64, generator=torch.Generator().manual_seed(2 + rank)).to(dev)

    def run(steps):
        inv = NullInversion(VideoP2PPipeline(unet), num_ddim_steps=steps)
        return inv.invert(x0, "", num_inner_steps=args.inner_steps, text_embeddings=ctx)

    for _ in range(args.warmup):
        run(2)
    torch.cuda.synchronize()
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        _, x_t, unc = run(args.ddim_steps)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        import torch.distributed as dist
        t = torch.tensor([elapsed], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    result = {
        "metric": "null-text inverted frames/sec (DDIM inversion + null-text optimisation, 512^2)",
        "value": round(args.frames * args.steps * world / elapsed, 5), "unit": "inverted frames/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 1), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": args.dtype,
        "data": "synthetic (random-init SD-1.5-geometry UNet3D, random text embeddings, x_0~N(0,1))",
        "config": {"workload": f"official-mode NullInversion.invert, {args.frames} frames 512^2, "
                               f"{args.ddim_steps} DDIM steps x {args.inner_steps} Adam iterations (max)",
                   "frames": args.frames, "ddim_steps": args.ddim_steps, "inner_steps": args.inner_steps,
                   "parallelism": f"clip-parallel x{world}"},
        "output_finite": bool(torch.isfinite(x_t).all().item()) and all(bool(torch.isfinite(u).all()) for u in unc),
    }
    if rank == 0:
        print(json.dumps(result), flush=True)


def _heartbeat(period=30.0):
    """A line on stderr every `period` s, so a long run (first use of new conv shapes, 24 frames) is
    never mistaken for a hung one."""
    import threading

    def beat():
        t0 = time.perf_counter()
        while True:
            time.sleep(period)
            print(f"[bench] running {time.perf_counter() - t0:.0f} s", file=sys.stderr, flush=True)
    threading.Thread(target=beat, daemon=True).start()


def main():
    args = parse()
    _heartbeat()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    torch.backends.cudnn.benchmark = bool(args.conv_find)
    if args.tuned:
        from vp2p.tuning import use_tuned_libraries
        use_tuned_libraries()
    if args.mode in ("nulltext", "k1long"):
        (nulltext_main if args.mode == "nulltext" else k1long_main)(args, world, rank, dev)
        if world > 1:
            import torch.distributed as dist
            dist.destroy_process_group()
        return

    import vp2p
    from vp2p import ops
    from vp2p.pipeline import VideoP2PPipeline
    from vp2p.tokenizer import SyntheticCLIPTokenizer
    from vp2p.unet3d import UNet3DConditionModel, init_random_

    dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    f = args.frames
    edit_name, edit_kind, (prompts, swap, blend, eq, cross, self_) = EDITS[args.edit]
    tok = SyntheticCLIPTokenizer()
    unet = init_random_(UNet3DConditionModel(), seed=0).to(dev, dtype).to(memory_format=torch.channels_last)
    unet.eval()
    ctrl = vp2p.make_controller(prompts, swap, {"default_": cross}, self_, blend, eq, tokenizer=tok,
                                num_steps=args.ddim_steps)
    vp2p.register_attention_control(type("Pipe", (), {"unet": unet})(), ctrl)
    g = torch.Generator().manual_seed(1)
    unc = torch.randn(1, 77, 768, generator=g)
    emb = torch.cat([unc, unc, torch.randn(2, 77, 768, generator=g)]).to(dev)
    frames_mode = args.shard == "frames" and world > 1
    x_T = torch.randn(1, 4, f, 64, 64,
                      generator=torch.Generator().manual_seed(2 if frames_mode else 2 + rank)).to(dev)
    pipe = VideoP2PPipeline(unet)
    shard = None
    if frames_mode:
        from vp2p.frame_parallel import FrameShard
        shard = FrameShard()
        x_T = shard.local(x_T, 2)
    f_run = x_T.shape[2]

    def edit():
        from vp2p.frame_parallel import frame_parallel
        ctrl.reset()
        with frame_parallel(shard):
            return pipe(prompts, f_run, latents=x_T, controller=ctrl, fast=True, text_embeddings=emb,
                        num_inference_steps=args.ddim_steps)

    def barrier():
        if world > 1:
            import torch.distributed as dist
            dist.barrier()

    with torch.no_grad():
        for _ in range(args.warmup):
            out = edit()
        torch.cuda.synchronize()
        timer = K1Timer(ops)
        with timer:
            timer.active = not args.no_k1_events
            barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                out = edit()
            torch.cuda.synchronize()
            barrier()
            t1 = time.perf_counter()
            timer.active = False
    elapsed = t1 - t0
    if world > 1:
        import torch.distributed as dist
        t = torch.tensor([elapsed], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    finite = bool(torch.isfinite(out).all().item())
    peak = PEAK_BF16_TFLOPS if dtype == torch.bfloat16 else PEAK_F32_TFLOPS
    roof = timer.summary(f, peak)
    result = {
        "metric": "edited frames/sec, 50-step DDIM P2P 512^2; attn MFMA util % of gfx950 peak",
        "value": round(f * args.steps * (1 if frames_mode else world) / elapsed, 4),
        "unit": "edited frames/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 2),
        "higher_is_better": True, "scaling": "strong" if frames_mode else "weak", "vs_baseline": None,
        "dtype": args.dtype, "data": "synthetic (random-init SD-1.5-geometry UNet3D, random text embeddings, x_T~N(0,1))",
        "config": {"workload": f"{edit_name} --fast: {edit_kind}, {f} frames 512^2, "
                               f"{args.ddim_steps}-step DDIM, UNet batch 4", "frames": f, "resolution": 512,
                   "ddim_steps": args.ddim_steps, "unet_batch": 4,
                   "parallelism": f"frame-sharded x{world} (RCCL)" if frames_mode else f"clip-parallel x{world}"},
        "roofline": roof,
        "output_finite": finite,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            result["cpu_baseline"] = cpu_baseline(f, args.ddim_steps, min(16, os.cpu_count() or 1))
        except Exception as e:  # keep the GPU line even if the host leg fails
            result["cpu_baseline"] = {"error": repr(e)}
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
