#!/usr/bin/env python
"""Benchmark: edited frames/s of a 50-step DDIM Video-P2P edit at 512^2 (BASELINE.json metric).

One "step" = one complete edit of one clip: 50 denoising steps of the UNet3D at batch 4
(2 prompts x CFG) with the P2P controller (AttentionRefine + LocalBlend + AttentionReweight of
configs/rabbit-jump-p2p.yaml), fast mode, DDIM eta = 0 -- configs[1] of BASELINE.json
("rabbit-jump-p2p 8f 512^2 on 1xMI355X bf16").  Synthetic data: random-init SD-1.5-geometry
UNet3D (seed 0, N(0, 0.02), attn_temp.to_out non-zero), random text embeddings standing in for
CLIP (seed 1; CLIP and VAE are excluded from the metric), x_T ~ N(0, 1) (seed 2).

Multi-GPU: ``python bench.py --gpus N`` starts N rank processes itself (a torchrun child, launched
before this process touches the GPU); under an external torchrun it reads RANK / WORLD_SIZE.  The
default ``--shard frames`` runs ONE clip over all ranks (frame_parallel.EditLayout): the CFG halves
on two rank groups, the frames sharded inside each half, RCCL carrying the frame-0 hidden-state
scatter + all-gather, the 5-D GroupNorm statistics and the attn_temp all-to-all.  ``--scale weak``
(default): the clip has 8 x N frames, so every rank keeps the N = 1 edit's per-forward work (32
images) -- frame-sharded weak scaling, the north star's "frames sharded across 1-8 GPUs" at the
bench's per-GPU size; the 8-frame clip over the same N ranks (strong scaling: 2 frames per rank at
N = 8, where the small per-launch work bounds it) is the secondary ``strong_scaling``
field, ``--scale strong`` makes it the headline.  value = clip frames / max-over-ranks wall time.
``--shard clips``: every rank edits its own clip, no collective; also reported as ``clip_parallel``.

The JSON line carries, measured live with HIP events on the launch stream inside the timed region:
``roofline`` for K1 (frame attention, the dominant MFMA-bound kernel: its res-64 launches),
``attention`` (K2 / K3 HBM rates and the aggregate attention MFMA utilisation over every K1/K2/K3
launch), plus -- at N = 1 -- the 50-step DDIM inversion rate, a reference-precision fp32 edit and
the CPU baseline (the oracle's fp32 UNet on the host cores, bounded sample, extrapolated).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "video-p2p_amd"))

import torch  # noqa: E402  (importing torch does not initialise the GPU)

PEAK_BF16_TFLOPS = 2500.0      # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
PEAK_F32_TFLOPS = 157.3        # dense fp32 MFMA
PEAK_HBM_GBS = 8000.0
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
    ap.add_argument("--no-events", "--no-k1-events", dest="no_events", action="store_true",
                    help="do not bracket the attention launches with HIP events")
    ap.add_argument("--scale", default="weak", choices=["weak", "strong"],
                    help="frame-sharded N > 1: weak = ONE clip of frames x N frames sharded over the N ranks "
                         "(every rank keeps the N = 1 edit's 32 images per UNet forward); strong = the "
                         "frames-frame clip itself (reported as the strong_scaling secondary either way)")
    ap.add_argument("--graphs", type=int, default=0,
                    help="1: replay each denoising step as a captured HIP graph (one process only; bit-equal)")
    ap.add_argument("--extras", default="auto", choices=["auto", "none", "all"],
                    help="secondary lines: inversion + fp32 edit (N = 1), clip-parallel (N > 1); auto = those")
    ap.add_argument("--mode", default="edit", choices=["edit", "nulltext", "k1long", "selftest"],
                    help="edit: the P2P edit (BASELINE metric, configs[1]); nulltext: official-mode inversion "
                         "(DDIM inversion + null-text optimisation, configs[3]), one step = one inversion; "
                         "k1long: configs[4], the FrameAttention of one UNet forward over a --long-frames clip "
                         "at 768^2, frames sharded over the ranks; selftest: the launcher and the rank "
                         "layout's collectives on the CPU (gloo), no GPU")
    ap.add_argument("--long-frames", type=int, default=128, help="k1long: frames of the clip")
    ap.add_argument("--conv-find", type=int, default=0,
                    help="1: run MIOpen's solver search per new conv shape (torch.backends.cudnn.benchmark; slow "
                         "warmup); 0 (default): immediate mode, which takes the tuned solvers recorded in the "
                         "in-tree database miopen_db/ (tools/miopen_tune.py)")
    ap.add_argument("--tuned", type=int, default=1,
                    help="1 (default): in-tree tuned MIOpen database (vp2p.tuning); 0: library heuristics")
    ap.add_argument("--inner-steps", type=int, default=10, help="null-text Adam iterations per DDIM step")
    ap.add_argument("--shard", default="frames", choices=["frames", "clips"],
                    help="frames (default): one clip over all ranks (CFG split x frame sharding; --scale picks "
                         "whether the headline clip grows with N); clips: every rank edits its own clip (no "
                         "collective)")
    return ap.parse_args()


# -- launcher -------------------------------------------------------------------------------------------
def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int, argv) -> int:
    """Start ``n`` rank processes of this script under torchrun (a CHILD process: this one has not
    touched the GPU and never execs) and return the launcher's exit code."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


# -- live kernel timing -----------------------------------------------------------------------------------
class AttnTimer:
    """Brackets every attention launch (K1 frame, K2 cross + P2P, K3 temporal) with HIP events on
    the launch stream while ``active``; ``summary`` turns them into algorithmic rates."""

    NAMES = ("frame_attention", "cross_attention_p2p", "temporal_attention_p2p")

    def __init__(self, ops, enabled=True):
        self.ops, self.enabled = ops, enabled
        self.orig = {n: getattr(ops, n) for n in self.NAMES}
        self.events = {n: [] for n in self.NAMES}
        self.active = False

    def __enter__(self):
        for name in self.NAMES:
            orig = self.orig[name]

            def wrapped(q, k, v, frames, heads, *a, _orig=orig, _name=name, **kw):
                if not (self.active and self.enabled):
                    return _orig(q, k, v, frames, heads, *a, **kw)
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                out = _orig(q, k, v, frames, heads, *a, **kw)
                e.record()
                self.events[_name].append((s, e, tuple(q.shape), tuple(k.shape), frames, q.element_size()))
                return out
            setattr(self.ops, name, wrapped)
        return self

    def __exit__(self, *exc):
        for name, fn in self.orig.items():
            setattr(self.ops, name, fn)

    @staticmethod
    def _work(name, qs, ks, frames, esz):
        """(algorithmic FLOP, algorithmic HBM bytes) of one launch."""
        Bf, N, C = qs
        B = Bf // frames
        if name == "frame_attention":       # QK^T + PV against frame-0 K/V; Q, O + frame-0 K, V once
            Nk = ks[1]
            return 4.0 * Bf * N * Nk * C, esz * (2 * Bf * N * C + 2 * B * Nk * C)
        if name == "cross_attention_p2p":   # 77 keys; Q in, O out, K/V once per batch row
            Nk = ks[1]
            return 4.0 * Bf * N * Nk * C, esz * (2 * Bf * N * C + 2 * B * Nk * C)
        # temporal: f x f per token; Q, K, V in, O out
        return 4.0 * Bf * N * frames * C, esz * 4 * Bf * N * C

    def summary(self, peak):
        if not any(self.events.values()):
            return None, None
        stats = {}
        tot_flop = tot_ms = 0.0
        for name, evs in self.events.items():
            if not evs:
                continue
            ms = [s.elapsed_time(e) for s, e, *_ in evs]
            flop = sum(self._work(name, qs, ks, f, esz)[0] for _, _, qs, ks, f, esz in evs)
            tot_flop += flop
            tot_ms += sum(ms)
            # the largest-token launches (res-64 at 512^2) are the headline shape of each kernel
            top = max(qs[1] for _, _, qs, *_ in evs)
            sel = [(m, ev) for m, ev in zip(ms, evs) if ev[2][1] == top]
            avg_ms = sum(m for m, _ in sel) / len(sel)
            f1, b1 = self._work(name, sel[0][1][2], sel[0][1][3], sel[0][1][4], sel[0][1][5])
            stats[name] = {"launches": len(evs), "time_ms": round(sum(ms), 2), "tokens": top,
                           "avg_ms": round(avg_ms, 4), "flop_per_launch": f1, "bytes_per_launch": b1,
                           "tflops": round(f1 / avg_ms / 1e9, 1), "gbs": round(b1 / avg_ms / 1e6, 1),
                           "shape": list(sel[0][1][2])}
        k1 = stats.get("frame_attention")
        roof = None
        if k1:
            traffic, src = _pmc_traffic(k1["shape"])
            roof = {"bound": "mfma", "achieved": k1["tflops"], "peak": peak, "unit": "TFLOP/s",
                    "frac": round(k1["tflops"] / peak, 4), "traffic": traffic, "traffic_unit": "bytes/launch",
                    "traffic_source": src, "algorithmic_bytes": k1["bytes_per_launch"],
                    "kernel": "vp2p::frame_attn_kernel_pp<2,8> (res-64 FrameAttention, software-pipelined, folded max)",
                    "launches": sum(1 for ev in self.events["frame_attention"] if ev[2][1] == k1["tokens"]),
                    "avg_ms": k1["avg_ms"], "flops_per_launch": k1["flop_per_launch"], "shape": k1["shape"]}
        attn = {"mfma_util": round(tot_flop / (tot_ms / 1e3) / 1e12 / peak, 4),
                "flop_per_edit_step_total": tot_flop, "kernel_ms_total": round(tot_ms, 2)}
        for key, name in (("k2_cross", "cross_attention_p2p"), ("k3_temporal", "temporal_attention_p2p")):
            if name in stats:
                st = stats[name]
                attn[key] = {"bound": "hbm", "achieved_gbs": st["gbs"], "peak_gbs": PEAK_HBM_GBS,
                             "frac": round(st["gbs"] / PEAK_HBM_GBS, 4), "avg_ms": st["avg_ms"],
                             "bytes_per_launch": st["bytes_per_launch"], "shape": st["shape"],
                             "launches": st["launches"]}
        if k1:
            attn["k1_frame"] = {"tflops": k1["tflops"], "frac": round(k1["tflops"] / peak, 4)}
        return roof, attn


TRAFFIC_FILE = os.path.join(ROOT, "profiles", "k1_pmc_traffic.json")


def _pmc_traffic(shape):
    """HBM bytes per K1 launch from committed rocprofv3 --pmc passes (FETCH_SIZE x2 per the gfx950
    correction, + WRITE_SIZE; tools/pmc_traffic.py) -- only when they were taken on this exact
    launch shape; otherwise None (the counters are not readable from inside the process)."""
    try:
        with open(TRAFFIC_FILE) as fh:
            d = json.load(fh)
        if list(d.get("shape", [])) != list(shape):
            return None, f"no PMC pass for shape {list(shape)} (profiles/k1_pmc_traffic.json is {d.get('shape')})"
        return d["bytes_per_launch"], os.path.relpath(TRAFFIC_FILE, ROOT) + " (" + d["how"] + ")"
    except (OSError, KeyError, ValueError):
        return None, None


# -- CPU baseline -----------------------------------------------------------------------------------------
def cpu_baseline(frames, ddim_steps, sample_frames=2):
    """The oracle's fp32 CPU UNet (oracle/unet_ref.py: the reference math, pinned to the reference's
    own model files), timed on this host's CPU share on a bounded sample (~30 s) and extrapolated:

    * the edit: ONE complete UNet forward of the edit (B = 4, every layer: 16 transformer blocks with
      the rabbit controller, 22 resnets, the up/down-sample convs) on ``sample_frames`` frames,
      x frames/sample_frames x ddim_steps (the headline unit, edited frames/s);
    * the inversion: one B = 1 forward (DummyController hook), x frames/sample_frames x ddim_steps;
    * per-layer attention: the reference's three attention ops alone at every
      attention resolution of the edit forward (B = 4, ``sample_frames`` frames): FrameAttention
      (attention.py:273-329), the hooked attn2 with the controller and attn_temp
      (ptp_utils.py:196-221), projections included, one call each.

    Every per-frame cost is linear in the frame count (frame attention reads frame 0's K/V; the
    temporal f x f attention is < 0.1% of the FLOPs).  Threads: torch's intra-op pool, i.e. the
    box's OMP_NUM_THREADS (the GPU box allots 16 host threads per GPU; nproc reports the whole host)."""
    from oracle import p2p_oracle as O
    from oracle import unet_ref
    from vp2p.tokenizer import SyntheticCLIPTokenizer
    from vp2p.unet3d import UNet3DConditionModel, init_random_
    threads = torch.get_num_threads()
    prompts, swap, blend, eq, cross, self_ = RABBIT
    ctrl = O.EditController(prompts, swap, {"default_": cross}, self_, SyntheticCLIPTokenizer(),
                            blend_words=blend, eq_params=eq)
    sd = init_random_(UNet3DConditionModel(), seed=0).state_dict()
    g = torch.Generator().manual_seed(3)
    x = torch.randn(4, 4, sample_frames, 64, 64, generator=g)
    ctx = torch.randn(4, 77, 768, generator=g)
    scale = frames / sample_frames * ddim_steps
    with torch.no_grad():
        t0 = time.perf_counter()
        unet_ref.unet_forward(sd, x, 981, ctx, ctrl)
        t_fwd = time.perf_counter() - t0
        t0 = time.perf_counter()
        unet_ref.unet_forward(sd, x[:1], 981, ctx[2:3])
        t_inv = time.perf_counter() - t0
        ctrl = O.EditController(prompts, swap, {"default_": cross}, self_, SyntheticCLIPTokenizer(),
                                blend_words=blend, eq_params=eq)
        layers = {}
        for res, p, (hw, C) in (("res64", "down_blocks.0.attentions.0.", (4096, 320)),
                                ("res32", "down_blocks.1.attentions.0.", (1024, 640)),
                                ("res16", "down_blocks.2.attentions.0.", (256, 1280)),
                                ("res8", "mid_block.attentions.0.", (64, 1280))):
            q = p + "transformer_blocks.0."
            xt = torch.randn(4 * sample_frames, hw, C, generator=g)
            ms = {}
            t0 = time.perf_counter()
            unet_ref.frame_attention(sd, q + "attn1.", xt, sample_frames)
            ms["frame_attn"] = (time.perf_counter() - t0) * 1e3
            t0 = time.perf_counter()
            unet_ref.hooked(sd, q + "attn2.", xt, ctx.repeat_interleave(sample_frames, 0), ctrl, "down")
            ms["cross_attn_p2p"] = (time.perf_counter() - t0) * 1e3
            xtt = xt.reshape(4, sample_frames, hw, C).permute(0, 2, 1, 3).reshape(4 * hw, sample_frames, C)
            t0 = time.perf_counter()
            unet_ref.hooked(sd, q + "attn_temp.", xtt, None, ctrl, "down")
            ms["temporal_attn_p2p"] = (time.perf_counter() - t0) * 1e3
            layers[res] = {k: round(v, 1) for k, v in ms.items()}
    t_edit = t_fwd * scale
    return {"value": round(frames / t_edit, 6), "unit": "edited frames/s", "cores": threads, "kind": "port",
            "sample": (f"oracle/unet_ref.py fp32 (pinned to tuneavideo's model files): one full UNet3D forward of the "
                       f"edit (B=4, {sample_frames} frames, 512^2, rabbit controller) timed once ({t_fwd:.1f} s), "
                       f"x{frames / sample_frames:g} frames x {ddim_steps} steps (extrapolated)"),
            "inversion": {"value": round(frames / (t_inv * scale), 6), "unit": "inverted frames/s",
                          "sample": f"one B=1 forward on {sample_frames} frames ({t_inv:.1f} s), extrapolated alike"},
            "attention_layer_ms": {"shape": f"B=4, {sample_frames} frames, one call per op (projections included)",
                                   **layers},
            "torch_threads": threads, "nproc": os.cpu_count(), "cpu_model": _cpu_model(),
            "cores_note": "torch intra-op threads = the box's OMP_NUM_THREADS (16 host threads per GPU on the "
                          "gpurun box); nproc counts the whole host"}


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


# -- other modes ----------------------------------------------------------------------------------------
def k1long_main(args, world, rank, dev):
    """configs[4] of BASELINE.json: sparse-causal (first-frame K/V) attention of a 128-frame 768^2
    clip, sharded by frames over the ranks.  One step = every attn1 call of one UNet forward at
    UNet batch 4 (5 blocks at 96^2 tokens / C 320, 5 at 48^2 / 640, 5 at 24^2 / 1280, 1 at 12^2 / 1280):
    per call rank 0 (owner of frame 0) broadcasts the frame-0 normed hidden state (B, HW, C) over
    RCCL, every rank projects frame 0's K|V and runs K1 on its f/G frames.  Synthetic bf16."""
    import torch.distributed as dist
    import torch.nn.functional as F
    from vp2p import ops
    B, heads, f = 4, 8, args.long_frames
    if f % world:
        raise SystemExit(f"--long-frames {f} does not split over {world} ranks")
    fl = f // world
    levels = [(96 * 96, 320, 5), (48 * 48, 640, 5), (24 * 24, 1280, 5), (12 * 12, 1280, 1)]
    g = torch.Generator(device=dev).manual_seed(3 + rank)
    bufs = []
    for hw, C, n in levels:
        # q as the to_q GEMM hands it to K1 (scale * log2 e folded in: FrameAttention.forward)
        q = (torch.randn(B * fl, hw, C, device=dev, generator=g) * ops.frame_query_scale(C // heads)).bfloat16()
        x0 = torch.randn(B, hw, C, device=dev, dtype=torch.bfloat16, generator=g)
        wkv = torch.randn(2 * C, C, device=dev, dtype=torch.bfloat16, generator=g) * C ** -0.5
        bufs.append((q, x0, wkv, torch.empty_like(q), C, n))

    def step():
        for q, x0, wkv, out, C, n in bufs:
            for _ in range(n):
                if world > 1:
                    dist.broadcast(x0, src=0)
                kv = F.linear(x0, wkv)
                ops.frame_attention(q, kv[..., :C], kv[..., C:], fl, heads, out=out, q_prescaled=True)

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
    elapsed = _max_over_ranks(time.perf_counter() - t0, world, dev)
    flops = sum(4.0 * B * f * hw * hw * C * n for hw, C, n in levels)
    result = {
        "metric": "sparse-causal attention TFLOP/s, 768^2 x 128-frame clip (K1 + RCCL frame-0 hidden broadcast)",
        "value": round(flops * args.steps / elapsed / 1e12, 1), "unit": "TFLOP/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 2), "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "bf16", "data": "synthetic (random bf16 q / frame-0 hidden / K|V weights)",
        "config": {"workload": f"attn1 of one UNet forward, {f} frames 768^2, UNet batch {B}, frame-sharded x{world}",
                   "frames": f, "resolution": 768, "unet_batch": B, "parallelism": f"frame-sharded x{world} (RCCL)"},
        "frames_per_s": round(f * args.steps / elapsed, 2),
        "roofline": {"bound": "mfma", "achieved": round(flops / world * args.steps / elapsed / 1e12, 1),
                     "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                     "frac": round(flops / world * args.steps / elapsed / 1e12 / PEAK_BF16_TFLOPS, 4),
                     "note": "per-GPU K1 algorithmic FLOP rate including the broadcast and K|V projection time"},
    }
    if rank == 0:
        print(json.dumps(result), flush=True)


def nulltext_main(args, world, rank, dev, quiet=False):
    """configs[3] of BASELINE.json: NullInversion.invert (run_videop2p.py:614-624) of an 8-frame 512^2
    clip: 50 DDIM-inversion steps, then per step one conditional forward, up to --inner-steps
    forward+backward Adam iterations (random weights never reach the early-stop epsilon, so always
    the maximum, the reference's worst case) and one guided step (B=2).  Over ranks: ``--shard frames``
    (default) shards ONE clip's frames -- forward and backward exchanges, the embedding gradient
    averaged before every Adam step (frame_parallel) -- ``--shard clips`` runs a clip per rank."""
    from vp2p.frame_parallel import FrameShard, frame_parallel
    from vp2p.pipeline import NullInversion, VideoP2PPipeline
    from vp2p.unet3d import UNet3DConditionModel, init_random_
    dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    unet = init_random_(UNet3DConditionModel(), seed=0).to(dev, dtype).to(memory_format=torch.channels_last)
    unet.eval()
    g = torch.Generator().manual_seed(1)
    ctx = torch.randn(2, 77, 768, generator=g).to(dev)
    frames_mode = args.shard == "frames" and world > 1
    shard = FrameShard() if frames_mode else None
    x0 = torch.randn(1, 4, args.frames, 64, 64,
                     generator=torch.Generator().manual_seed(2 + (0 if frames_mode else rank))).to(dev)
    if shard is not None:
        x0 = shard.local(x0, 2)

    def run(steps):
        with frame_parallel(shard):
            inv = NullInversion(VideoP2PPipeline(unet), num_ddim_steps=steps)
            return inv.invert(x0, "", num_inner_steps=args.inner_steps, text_embeddings=ctx)

    for _ in range(args.warmup):
        run(2)
    torch.cuda.synchronize()
    _barrier(world)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        _, x_t, unc = run(args.ddim_steps)
    torch.cuda.synchronize()
    _barrier(world)
    elapsed = _max_over_ranks(time.perf_counter() - t0, world, dev)
    del unet
    torch.cuda.empty_cache()
    result = {
        "metric": "null-text inverted frames/sec (DDIM inversion + null-text optimisation, 512^2)",
        "value": round(args.frames * args.steps * (1 if frames_mode else world) / elapsed, 5),
        "unit": "inverted frames/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 1), "higher_is_better": True,
        "scaling": "strong" if frames_mode else "weak",
        "vs_baseline": None, "dtype": args.dtype,
        "data": "synthetic (random-init SD-1.5-geometry UNet3D, random text embeddings, x_0~N(0,1))",
        "config": {"workload": f"official-mode NullInversion.invert, {args.frames} frames 512^2, "
                               f"{args.ddim_steps} DDIM steps x {args.inner_steps} Adam iterations (max)",
                   "frames": args.frames, "ddim_steps": args.ddim_steps, "inner_steps": args.inner_steps,
                   "parallelism": f"frame-sharded x{world} (RCCL)" if frames_mode else f"clip-parallel x{world}"},
        "output_finite": bool(torch.isfinite(x_t).all().item()) and all(bool(torch.isfinite(u).all()) for u in unc),
    }
    if rank == 0 and not quiet:
        print(json.dumps(result), flush=True)
    return result


def selftest_main(args, world, rank):
    """CPU (gloo) rehearsal of the multi-rank path: the launcher brought up ``world`` ranks; build the
    EditLayout and run each of its exchanges on CPU tensors against the single-rank answer."""
    import torch.distributed as dist
    from vp2p.frame_parallel import EditLayout
    lay = EditLayout()
    P, f, N, C = 2, 8, 16, 6
    g = torch.Generator().manual_seed(7)
    full = torch.randn(2 * P, 4, f, 8, 8, generator=g)              # [uncond x P, cond x P] noise
    fl = lay.frames_local(f)
    half = lay.half if lay.cfg_split else None
    rows = full if half is None else full[half * P:(half + 1) * P]
    mine = lay.local(rows, 2)
    got = lay.gather_cfg(mine)
    want = lay.local(full, 2) if half is not None else mine
    ok = torch.equal(got, want)
    if lay.frames is not None:                                          # frame-0 hidden broadcast
        x0 = torch.full((2, N, C), float(lay.rank)) if lay.frames.rank else torch.full((2, N, C), -1.0)
        lay.frames.broadcast_(x0)
        ok &= bool((x0 == -1.0).all())
        x = torch.randn(2 * fl, N, C, generator=torch.Generator().manual_seed(11 + lay.frame_rank))
        ok &= torch.equal(lay.frames.to_frames(lay.frames.to_tokens(x, 2), 2), x)
    t = torch.tensor([float(ok)])
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    if rank == 0:
        print(json.dumps({"selftest": "ok" if t.item() == 1.0 else "FAILED", "world": world,
                          "layout": lay.describe(), "frames_local": fl}), flush=True)
    if t.item() != 1.0:
        raise SystemExit(1)


# -- helpers ----------------------------------------------------------------------------------------------
def _barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def _max_over_ranks(x: float, world: int, dev) -> float:
    if world == 1:
        return x
    import torch.distributed as dist
    t = torch.tensor([x], device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


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


class Edit:
    """One edit configuration (model, controller, inputs) ready to run under a layout."""

    def __init__(self, args, dev, dtype, layout=None, seed_offset=0):
        import vp2p
        from vp2p.pipeline import VideoP2PPipeline
        from vp2p.tokenizer import SyntheticCLIPTokenizer
        from vp2p.unet3d import UNet3DConditionModel, init_random_
        self.f = args.frames
        self.steps = args.ddim_steps
        name, kind, (prompts, swap, blend, eq, cross, self_) = EDITS[args.edit]
        self.name, self.kind, self.prompts = name, kind, prompts
        self.unet = init_random_(UNet3DConditionModel(), seed=0).to(dev, dtype).to(memory_format=torch.channels_last)
        self.unet.eval()
        self.ctrl = vp2p.make_controller(prompts, swap, {"default_": cross}, self_, blend, eq,
                                         tokenizer=SyntheticCLIPTokenizer(), num_steps=args.ddim_steps)
        vp2p.register_attention_control(type("Pipe", (), {"unet": self.unet})(), self.ctrl)
        g = torch.Generator().manual_seed(1)
        unc = torch.randn(1, 77, 768, generator=g)
        self.emb = torch.cat([unc, unc, torch.randn(2, 77, 768, generator=g)]).to(dev)
        x_T = torch.randn(1, 4, self.f, 64, 64, generator=torch.Generator().manual_seed(2 + seed_offset)).to(dev)
        self.layout = layout
        self.x_T = layout.local(x_T, 2) if layout is not None else x_T
        self.pipe = VideoP2PPipeline(self.unet)
        self.graphs = bool(getattr(args, "graphs", 0)) and layout is None

    def __call__(self):
        from vp2p.frame_parallel import frame_parallel
        self.ctrl.reset()
        with frame_parallel(self.layout):
            return self.pipe(self.prompts, self.x_T.shape[2], latents=self.x_T, controller=self.ctrl, fast=True,
                             text_embeddings=self.emb, num_inference_steps=self.steps, graphs=self.graphs)


def _time_edits(edit, warmup, steps, world, dev, timer=None):
    for _ in range(warmup):
        out = edit()
    torch.cuda.synchronize()
    _barrier(world)
    torch.cuda.synchronize()
    if timer is not None:
        timer.active = True
    t0 = time.perf_counter()
    for _ in range(steps):
        out = edit()
    torch.cuda.synchronize()
    _barrier(world)
    t1 = time.perf_counter()
    if timer is not None:
        timer.active = False
    return _max_over_ranks(t1 - t0, world, dev), out


def inversion_line(edit, dev, reps=2):
    """Fast-mode DDIM inversion (NullInversion.invert_, run_videop2p.py:626-635 / ddim_loop :557-567):
    50 UNet forwards at batch 1 (DummyController), reported separately."""
    import vp2p
    from vp2p.pipeline import NullInversion, VideoP2PPipeline
    unet = edit.unet
    x0 = torch.randn(1, 4, edit.f, 64, 64, generator=torch.Generator().manual_seed(4)).to(dev)
    ctx = edit.emb[[0, 2]].contiguous()                   # [uncond, cond of the source prompt]
    inv = NullInversion(VideoP2PPipeline(unet), num_ddim_steps=edit.steps)
    inv.invert_(x0, "", text_embeddings=ctx)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        _, x_t, _ = inv.invert_(x0, "", text_embeddings=ctx)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    vp2p.register_attention_control(type("Pipe", (), {"unet": unet})(), edit.ctrl)   # back to the edit
    return {"metric": f"inverted frames/sec ({edit.steps}-step DDIM inversion, batch 1, 512^2)",
            "value": round(edit.f / dt, 4), "unit": "inverted frames/s", "ms_per_inversion": round(dt * 1e3, 1),
            "output_finite": bool(torch.isfinite(x_t).all().item())}


def vae_line(latents, dev, dtype, reps=2):
    """VAE decode of the edit's output latents (TuneAVideoPipeline.decode_latents,
    pipeline_tuneavideo.py:239-256: (b f) frames in batches of 4, vp2p.vae on K7 + MIOpen), outside
    the headline metric (the reference's edit timing also stops at the latents)."""
    from vp2p.vae import AutoencoderKL, decode_latents, init_vae_random_
    vae = init_vae_random_(AutoencoderKL(), seed=0).to(dev, dtype).to(memory_format=torch.channels_last).eval()
    video = decode_latents(vae, latents)                 # first use: MIOpen picks / loads its kernels
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        video = decode_latents(vae, latents)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    n = latents.shape[0] * latents.shape[2]
    return {"metric": "decoded frames/sec (VAE decode of the edited latents, 512^2)", "value": round(n / dt, 3),
            "unit": "decoded frames/s", "frames": n, "ms_per_clip": round(dt * 1e3, 1), "dtype": str(dtype).split(".")[-1],
            "output_finite": bool(torch.isfinite(video).all().item())}


def main():
    args = parse()
    if args.graphs:
        args.no_events = True          # replays bypass the Python launch wrappers the event timer hooks
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: launch with matching counts")
    if args.mode == "selftest":
        import torch.distributed as dist
        if world > 1:
            dist.init_process_group("gloo")
        try:
            selftest_main(args, world, rank)
        finally:
            if world > 1:
                dist.destroy_process_group()
        return
    _heartbeat()
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
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

    from vp2p import ops
    dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    peak = PEAK_BF16_TFLOPS if dtype == torch.bfloat16 else PEAK_F32_TFLOPS
    frames_mode = args.shard == "frames" and world > 1
    layout = None
    f1 = args.frames                                    # the clip of the N = 1 workload (configs[1]: 8)
    weak_frames = frames_mode and args.scale == "weak"
    if weak_frames:
        # weak frame scaling: one clip of f1 * N frames, sharded (CFG split x frame shards), so each
        # rank runs the N = 1 edit's per-forward work (B2 x 2 f1 frames = B4 x f1 images) and every
        # cross-frame exchange of the layout carries real traffic
        args.frames = f1 * world
    layout = None
    if frames_mode:
        from vp2p.frame_parallel import EditLayout
        layout = EditLayout()
    edit = Edit(args, dev, dtype, layout, seed_offset=0 if frames_mode else rank)
    with torch.no_grad():
        with AttnTimer(ops, enabled=not args.no_events) as timer:
            elapsed, out = _time_edits(edit, args.warmup, args.steps, world, dev, timer)
    finite = bool(torch.isfinite(out).all().item())
    roof, attn = timer.summary(peak)
    f = args.frames
    result = {
        "metric": "edited frames/sec, 50-step DDIM P2P 512^2; attn MFMA util % of gfx950 peak",
        "value": round(f * args.steps * (1 if frames_mode else world) / elapsed, 4),
        "unit": "edited frames/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 2),
        "higher_is_better": True, "scaling": "strong" if (frames_mode and not weak_frames) else "weak",
        "vs_baseline": None,
        "dtype": args.dtype, "data": "synthetic (random-init SD-1.5-geometry UNet3D, random text embeddings, x_T~N(0,1))",
        "config": {"workload": f"{edit.name} --fast: {edit.kind}, {f} frames 512^2, "
                               f"{args.ddim_steps}-step DDIM, UNet batch 4", "frames": f, "resolution": 512,
                   "ddim_steps": args.ddim_steps, "unet_batch": 4,
                   "parallelism": (layout.describe() + " (RCCL)") if frames_mode else f"clip-parallel x{world}"},
        "roofline": roof,
        "attention": attn,
        "output_finite": finite,
    }
    extras = args.extras != "none"
    with torch.no_grad():
        if extras and world > 1 and frames_mode and weak_frames:
            # secondary: strong frame scaling -- the N = 1 clip (f1 frames) sharded over the N ranks
            del edit
            torch.cuda.empty_cache()
            s_args = argparse.Namespace(**{**vars(args), "frames": f1})
            s_lay = EditLayout()
            strong = Edit(s_args, dev, dtype, s_lay, seed_offset=0)
            t_s, _ = _time_edits(strong, 1, 1, world, dev)
            result["strong_scaling"] = {"value": round(f1 / t_s, 4), "ms_per_step": round(t_s * 1e3, 2),
                                        "frames": f1, "scaling": "strong",
                                        "parallelism": s_lay.describe() + " (RCCL)"}
            del strong
        if extras and world > 1 and frames_mode:
            # secondary: every rank edits its own N = 1 clip (no collective), one timed edit
            c_args = argparse.Namespace(**{**vars(args), "frames": f1})
            clip = Edit(c_args, dev, dtype, None, seed_offset=rank)
            t_clip, _ = _time_edits(clip, 1, 1, world, dev)
            result["clip_parallel"] = {"value": round(f1 * world / t_clip, 4), "ms_per_step": round(t_clip * 1e3, 2),
                                       "scaling": "weak", "parallelism": f"clip-parallel x{world}"}
            del clip
        if extras and world == 1:
            result["inversion"] = inversion_line(edit, dev)
            result["vae_decode"] = vae_line(out, dev, dtype)
            if dtype == torch.bfloat16 and args.extras in ("auto", "all"):
                del edit
                torch.cuda.empty_cache()
                ref_args = argparse.Namespace(**{**vars(args), "dtype": "fp32"})
                e32 = Edit(ref_args, dev, torch.float32)
                with AttnTimer(ops, enabled=not args.no_events) as t32:
                    el32, out32 = _time_edits(e32, 1, 1, 1, dev, t32)
                r32, a32 = t32.summary(PEAK_F32_TFLOPS)
                result["fp32_edit"] = {"value": round(f / el32, 4), "unit": "edited frames/s",
                                       "ms_per_step": round(el32 * 1e3, 1), "dtype": "fp32",
                                       "note": "reference precision (run_videop2p.py:111-113 runs the UNet in fp32)",
                                       "k1_frac_of_fp32_peak": None if r32 is None else r32["frac"],
                                       "attn_mfma_util_fp32": None if a32 is None else a32["mfma_util"],
                                       "output_finite": bool(torch.isfinite(out32).all().item())}
                del e32
        if extras and (world == 1 or frames_mode):
            # secondary: configs[2] -- the penguin-run refine edit (seq_aligner mapper + LocalBlend +
            # Reweight), 24 frames, ONE clip frame-sharded over the N ranks (CFG split x frame shards):
            # strong scaling where the north star measures it; at N = 1 the single-GPU point of that curve
            edit = None
            torch.cuda.empty_cache()
            p_args = argparse.Namespace(**{**vars(args), "frames": 24, "edit": "penguin"})
            p_lay = EditLayout() if world > 1 else None
            peng = Edit(p_args, dev, dtype, p_lay, seed_offset=0)
            t_p, _ = _time_edits(peng, 1, 1, world, dev)
            result["strong_scaling_24f"] = {
                "value": round(24 / t_p, 4), "unit": "edited frames/s", "ms_per_step": round(t_p * 1e3, 2),
                "frames": 24, "scaling": "strong", "config": "configs[2]: " + peng.name + " --fast, " + peng.kind,
                "parallelism": (p_lay.describe() + " (RCCL)") if p_lay is not None else "single GPU"}
            del peng
            torch.cuda.empty_cache()
        if extras and world == 1:
            # secondary: configs[3] -- official mode, NullInversion.invert of an 8-frame clip (50 DDIM
            # inversion steps + 10 Adam iterations per step under autograd), one timed clip
            try:
                n_args = argparse.Namespace(**{**vars(args), "frames": f1, "steps": 1, "warmup": 1, "shard": "frames"})
                with torch.enable_grad():       # the Adam iterations differentiate the UNet
                    nt = nulltext_main(n_args, 1, rank, dev, quiet=True)
                result["nulltext"] = {k: nt[k] for k in ("metric", "value", "unit", "ms_per_step", "config", "output_finite")}
            except Exception as e:      # keep the headline line if the secondary fails
                result["nulltext"] = {"error": repr(e)}
            torch.cuda.empty_cache()
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            result["cpu_baseline"] = cpu_baseline(f, args.ddim_steps)
        except Exception as e:  # keep the GPU line even if the host leg fails
            result["cpu_baseline"] = {"error": repr(e)}
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
