"""CPU fp32 restatement of the tuneavideo UNet3D forward with the P2P hook.  TEST INFRASTRUCTURE
ONLY (importable by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg).

Functional form over a state dict (keys as tuneavideo checkpoints), written against the
reference's semantics:
  unet.py:279-414            time embedding, conv_in, down / mid / up wiring, conv_norm_out
  unet_blocks.py:125-589     block wiring, skip order, up-block concatenation
  resnet.py:11-205           inflated convs, 5-D GroupNorm (statistics over c/G x f x h x w)
  attention.py:90-329        Transformer3DModel / BasicTransformerBlock / FrameAttention
                             (first-frame K/V), the '(b f) d c -> (b d) f c' temporal rearrange
  ptp_utils.py:196-221       hooked attn2 / attn_temp with the numpy oracle controller
Dense layers use torch CPU fp32 (the reference's own ops); frame attention is chunked per
(batch*frame) slab instead of materialising the (B*f*h, HW, HW) score tensor.
"""
from __future__ import annotations

import math
from typing import Dict, Optional

import numpy as np
import torch
import torch.nn.functional as F

from . import p2p_oracle as O

HEADS = 8


def _conv_frames(x5: torch.Tensor, sd, p: str, stride: int = 1) -> torch.Tensor:
    """InflatedConv3d: Conv2d over '(b f)' (resnet.py:11-19)."""
    B, C, f, H, W = x5.shape
    w = sd[p + "weight"]
    y = F.conv2d(x5.permute(0, 2, 1, 3, 4).reshape(B * f, C, H, W), w, sd.get(p + "bias"),
                 stride=stride, padding=w.shape[-1] // 2)
    return y.reshape(B, f, *y.shape[1:]).permute(0, 2, 1, 3, 4)


def _gn(x, sd, p, eps):
    return F.group_norm(x, 32, sd[p + "weight"], sd[p + "bias"], eps)


def _lin(x, sd, p):
    return F.linear(x, sd[p + "weight"], sd.get(p + "bias"))


def _ln(x, sd, p):
    return F.layer_norm(x, (x.shape[-1],), sd[p + "weight"], sd[p + "bias"], 1e-5)


def resnet(sd, p, x5, temb, eps=1e-5):
    h = _conv_frames(F.silu(_gn(x5, sd, p + "norm1.", eps)), sd, p + "conv1.")
    h = h + _lin(F.silu(temb), sd, p + "time_emb_proj.")[:, :, None, None, None]
    h = _conv_frames(F.silu(_gn(h, sd, p + "norm2.", eps)), sd, p + "conv2.")
    sc = _conv_frames(x5, sd, p + "conv_shortcut.") if (p + "conv_shortcut.weight") in sd else x5
    return sc + h


def frame_attention(sd, p, x, f):
    """attention.py:273-329 on (B*f, N, C)."""
    Bf, N, C = x.shape
    B = Bf // f
    q = _lin(x, sd, p + "to_q.")
    x0 = x.reshape(B, f, N, C)[:, 0]
    k = _lin(x0, sd, p + "to_k.")
    v = _lin(x0, sd, p + "to_v.")
    d = C // HEADS
    out = torch.empty_like(q)
    for b in range(B):
        kb = k[b].reshape(N, HEADS, d).permute(1, 0, 2)
        vb = v[b].reshape(N, HEADS, d).permute(1, 0, 2)
        for fr in range(f):
            qb = q[b * f + fr].reshape(N, HEADS, d).permute(1, 0, 2)
            s = torch.softmax(torch.bmm(qb, kb.transpose(1, 2)) * (d ** -0.5), dim=-1)
            out[b * f + fr] = torch.bmm(s, vb).permute(1, 0, 2).reshape(N, C)
    return _lin(out, sd, p + "to_out.0.")


def hooked(sd, p, x, ctx, controller, place):
    """ptp_utils.py:196-221 (torch CPU fp32, global-max softmax, numpy oracle controller).  With no
    controller (the DummyController of :225-234) it stays in torch, so autograd can differentiate it."""
    is_cross = ctx is not None
    c = ctx if is_cross else x
    if controller is None:
        def heads(t):
            b, n, dim = t.shape
            return t.reshape(b, n, HEADS, dim // HEADS).permute(0, 2, 1, 3).reshape(b * HEADS, n, dim // HEADS)
        q, k, v = heads(_lin(x, sd, p + "to_q.")), heads(_lin(c, sd, p + "to_k.")), heads(_lin(c, sd, p + "to_v."))
        sim = torch.bmm(q, k.transpose(1, 2)) * (q.shape[-1] ** -0.5)
        e = torch.exp(sim - sim.max())
        out = torch.bmm(e / e.sum(-1, keepdim=True), v)
        bh, n, d = out.shape
        out = out.reshape(bh // HEADS, HEADS, n, d).permute(0, 2, 1, 3).reshape(bh // HEADS, n, HEADS * d)
        return _lin(out, sd, p + "to_out.0.")
    q = O.heads_to_batch(_lin(x, sd, p + "to_q.").numpy(), HEADS)
    k = O.heads_to_batch(_lin(c, sd, p + "to_k.").numpy(), HEADS)
    v = O.heads_to_batch(_lin(c, sd, p + "to_v.").numpy(), HEADS)
    sim = torch.bmm(torch.from_numpy(q), torch.from_numpy(k).transpose(1, 2)) * (q.shape[-1] ** -0.5)
    e = torch.exp(sim - sim.max())
    attn = (e / e.sum(-1, keepdim=True)).numpy()
    if controller is not None:
        attn = controller(attn, is_cross, place)
    out = torch.bmm(torch.from_numpy(np.ascontiguousarray(attn)), torch.from_numpy(v)).numpy()
    return _lin(torch.from_numpy(O.batch_to_heads(out, HEADS)), sd, p + "to_out.0.")


def transformer(sd, p, x5, ctx, controller, place):
    B, C, f, H, W = x5.shape
    x = x5.permute(0, 2, 1, 3, 4).reshape(B * f, C, H, W)
    res = x
    h = F.group_norm(x, 32, sd[p + "norm.weight"], sd[p + "norm.bias"], 1e-6)
    h = F.conv2d(h, sd[p + "proj_in.weight"], sd[p + "proj_in.bias"])
    t = h.permute(0, 2, 3, 1).reshape(B * f, H * W, C)
    q = p + "transformer_blocks.0."
    t = frame_attention(sd, q + "attn1.", _ln(t, sd, q + "norm1."), f) + t
    ctx_f = ctx.repeat_interleave(f, 0)                                   # attention.py:95
    t = hooked(sd, q + "attn2.", _ln(t, sd, q + "norm2."), ctx_f, controller, place) + t
    a, g = _lin(_ln(t, sd, q + "norm3."), sd, q + "ff.net.0.proj.").chunk(2, dim=-1)
    t = _lin(a * F.gelu(g), sd, q + "ff.net.2.") + t
    tt = t.reshape(B, f, H * W, C).permute(0, 2, 1, 3).reshape(B * H * W, f, C)   # '(b d) f c'
    tt = hooked(sd, q + "attn_temp.", _ln(tt, sd, q + "norm_temp."), None, controller, place) + tt
    t = tt.reshape(B, H * W, f, C).permute(0, 2, 1, 3).reshape(B * f, H * W, C)
    h = t.reshape(B * f, H, W, C).permute(0, 3, 1, 2)
    h = F.conv2d(h, sd[p + "proj_out.weight"], sd[p + "proj_out.bias"]) + res
    return h.reshape(B, f, C, H, W).permute(0, 2, 1, 3, 4)


def transformer_token_slice(sd, p, x5, ctx, tokens, dtype=torch.float64):
    """``transformer`` (Transformer3DModel.forward, attention.py:90-137, 233-270; plain attention =
    the DummyController hook in the finite regime) evaluated only at the spatial positions
    ``tokens`` (indices into H*W), for every frame: (B, C, f, len(tokens)).

    Exact for a long clip without computing all of it: GroupNorm statistics are per frame over all
    positions (computed in full), attn1 needs Q at the slice and frame 0's K/V at every position
    (attention.py:296-302), attn2 and the feed-forward are per position, and attn_temp mixes only the
    frames of one position (attention.py:262-268).  ``dtype``: arithmetic precision (float64 = an
    independent high-precision check of the fp32/bf16 kernels)."""
    B, C, f, H, W = x5.shape
    sd = {k: v.to(dtype) for k, v in sd.items()}
    tok = torch.as_tensor(tokens, dtype=torch.int64)
    S = tok.numel()
    G = 32
    xs = torch.empty(B, f, S, C, dtype=dtype)          # x at the slice: (b, f, s, c)
    hs = torch.empty(B, f, S, C, dtype=dtype)          # GroupNorm(x) at the slice
    h0 = torch.empty(B, H * W, C, dtype=dtype)         # GroupNorm(x) of frame 0, every position
    for b in range(B):
        for fr in range(f):
            xf = x5[b, :, fr].reshape(C, H * W).to(dtype)
            g = xf.reshape(G, -1)
            mean = g.mean(1, keepdim=True)
            var = g.var(1, unbiased=False, keepdim=True)
            hn = ((g - mean) / torch.sqrt(var + 1e-6)).reshape(C, H * W)
            hn = hn * sd[p + "norm.weight"][:, None] + sd[p + "norm.bias"][:, None]
            xs[b, fr] = xf[:, tok].T
            hs[b, fr] = hn[:, tok].T
            if fr == 0:
                h0[b] = hn.T
    w_in = sd[p + "proj_in.weight"].reshape(C, C)
    t = hs @ w_in.T + sd[p + "proj_in.bias"]            # (B, f, S, C)
    t0 = h0 @ w_in.T + sd[p + "proj_in.bias"]           # (B, HW, C): frame 0, every position
    q_ = p + "transformer_blocks.0."
    d = C // HEADS

    def lin(x, name):
        return F.linear(x, sd[name + "weight"], sd.get(name + "bias"))

    def ln(x, name):
        return F.layer_norm(x, (C,), sd[name + "weight"], sd[name + "bias"], 1e-5)

    def attend(q, k, v):
        """q (..., Nq, C), k/v (..., Nk, C): softmax(q k^T d^-1/2) v per head."""
        qh = q.reshape(*q.shape[:-1], HEADS, d).transpose(-2, -3)
        kh = k.reshape(*k.shape[:-1], HEADS, d).transpose(-2, -3)
        vh = v.reshape(*v.shape[:-1], HEADS, d).transpose(-2, -3)
        a = torch.softmax(qh @ kh.transpose(-1, -2) * d ** -0.5, dim=-1)
        o = (a @ vh).transpose(-2, -3)
        return o.reshape(*o.shape[:-2], C)

    a1 = q_ + "attn1."
    k0 = lin(ln(t0, q_ + "norm1."), a1 + "to_k.")                  # (B, HW, C)
    v0 = lin(ln(t0, q_ + "norm1."), a1 + "to_v.")
    qa = lin(ln(t, q_ + "norm1."), a1 + "to_q.")                   # (B, f, S, C)
    t = lin(attend(qa, k0[:, None], v0[:, None]), a1 + "to_out.0.") + t
    a2 = q_ + "attn2."
    c = ctx.to(dtype)[:, None]                                     # (B, 1, 77, D): repeated per frame
    t = lin(attend(lin(ln(t, q_ + "norm2."), a2 + "to_q."), lin(c, a2 + "to_k."), lin(c, a2 + "to_v.")),
            a2 + "to_out.0.") + t
    a, g = lin(ln(t, q_ + "norm3."), q_ + "ff.net.0.proj.").chunk(2, dim=-1)
    t = lin(a * F.gelu(g), q_ + "ff.net.2.") + t
    tt = t.transpose(1, 2)                                         # (B, S, f, C): '(b d) f c'
    n = ln(tt, q_ + "norm_temp.")
    at = q_ + "attn_temp."
    tt = lin(attend(lin(n, at + "to_q."), lin(n, at + "to_k."), lin(n, at + "to_v.")), at + "to_out.0.") + tt
    w_out = sd[p + "proj_out.weight"].reshape(C, C)
    y = tt @ w_out.T + sd[p + "proj_out.bias"] + xs.transpose(1, 2)     # (B, S, f, C)
    return y.permute(0, 3, 2, 1)


def timestep_embedding(t: torch.Tensor, dim: int = 320) -> torch.Tensor:
    half = dim // 2
    freqs = torch.exp(-math.log(10000) * torch.arange(half, dtype=torch.float32) / half)
    e = t[:, None].float() * freqs[None]
    return torch.cat([torch.cos(e), torch.sin(e)], dim=-1)   # flip_sin_to_cos=True


def unet_forward(sd: Dict[str, torch.Tensor], sample: torch.Tensor, timestep: int, ctx: torch.Tensor,
                 controller=None, n_down: int = 4, layers: int = 2) -> torch.Tensor:
    """sample (B, 4, f, H, W), ctx (B, 77, D) -> noise prediction (B, 4, f, H, W)."""
    sd = {k: v.float().cpu() for k, v in sd.items()}
    B = sample.shape[0]
    t = torch.full((B,), int(timestep), dtype=torch.int64)
    emb = _lin(F.silu(_lin(timestep_embedding(t, sd["conv_in.weight"].shape[0]), sd, "time_embedding.linear_1.")),
               sd, "time_embedding.linear_2.")
    x = _conv_frames(sample.float(), sd, "conv_in.")
    skips = [x]
    for i in range(n_down):
        p = f"down_blocks.{i}."
        for j in range(layers):
            x = resnet(sd, p + f"resnets.{j}.", x, emb)
            if (p + f"attentions.{j}.norm.weight") in sd:
                x = transformer(sd, p + f"attentions.{j}.", x, ctx, controller, "down")
            skips.append(x)
        if (p + "downsamplers.0.conv.weight") in sd:
            x = _conv_frames(x, sd, p + "downsamplers.0.conv.", stride=2)
            skips.append(x)
    x = resnet(sd, "mid_block.resnets.0.", x, emb)
    x = transformer(sd, "mid_block.attentions.0.", x, ctx, controller, "mid")
    x = resnet(sd, "mid_block.resnets.1.", x, emb)
    for i in range(n_down):
        p = f"up_blocks.{i}."
        for j in range(layers + 1):
            x = torch.cat([x, skips.pop()], dim=1)
            x = resnet(sd, p + f"resnets.{j}.", x, emb)
            if (p + f"attentions.{j}.norm.weight") in sd:
                x = transformer(sd, p + f"attentions.{j}.", x, ctx, controller, "up")
        if (p + "upsamplers.0.conv.weight") in sd:
            B_, C_, f_, H_, W_ = x.shape
            x = F.interpolate(x, scale_factor=(1.0, 2.0, 2.0), mode="nearest")
            x = _conv_frames(x, sd, p + "upsamplers.0.conv.")
    x = F.silu(F.group_norm(x, 32, sd["conv_norm_out.weight"], sd["conv_norm_out.bias"], 1e-5))
    return _conv_frames(x, sd, "conv_out.")


def _prev_step(ddim: "O.DDIM", eps: torch.Tensor, t: int, x: torch.Tensor) -> torch.Tensor:
    """NullInversion.prev_step (run_videop2p.py:445-453) in torch ops (differentiable)."""
    prev_t = t - ddim.num_train_timesteps // ddim.num_inference_steps
    a_t = torch.tensor(ddim.alphas_cumprod[t])
    a_prev = torch.tensor(ddim._ac(prev_t))
    x0 = (x - (1 - a_t) ** 0.5 * eps) / a_t ** 0.5
    return a_prev ** 0.5 * x0 + (1 - a_prev) ** 0.5 * eps


def null_optimization(sd, latents, uncond: torch.Tensor, cond: torch.Tensor, ddim: "O.DDIM",
                      num_inner_steps: int = 10, epsilon: float = 1e-5, guidance: float = 7.5):
    """NullInversion.null_optimization (run_videop2p.py:580-612) on the CPU fp32 UNet with torch
    autograd and torch's Adam.  latents: the DDIM-inversion list [x_0 .. x_T]; returns
    (per-step optimised unconditional embeddings, every inner loss, final latent)."""
    out, losses = [], []
    latent_cur = latents[-1]
    ts = [int(t) for t in ddim.timesteps]
    for i, t in enumerate(ts):
        uncond = uncond.clone().detach()
        uncond.requires_grad = True
        opt = torch.optim.Adam([uncond], lr=1e-2 * (1.0 - i / 100.0))
        latent_prev = latents[len(latents) - i - 2]
        with torch.no_grad():
            noise_cond = unet_forward(sd, latent_cur, t, cond)
        for _ in range(num_inner_steps):
            noise_uncond = unet_forward(sd, latent_cur, t, uncond)
            noise = noise_uncond + guidance * (noise_cond - noise_uncond)
            loss = F.mse_loss(_prev_step(ddim, noise, t, latent_cur), latent_prev)
            opt.zero_grad()
            loss.backward()
            opt.step()
            losses.append(loss.item())
            if losses[-1] < epsilon + i * 2e-5:
                break
        out.append(uncond[:1].detach())
        with torch.no_grad():
            noise = unet_forward(sd, torch.cat([latent_cur] * 2), t, torch.cat([uncond, cond]))
            u, c = noise.chunk(2)
            latent_cur = _prev_step(ddim, u + guidance * (c - u), t, latent_cur)
    return out, losses, latent_cur
