"""CPU fp32 restatement of diffusers 0.11.1 ``AutoencoderKL`` (the SD-1.5 VAE) over a state dict.
TEST INFRASTRUCTURE ONLY (imported by tests/ and bench.py's cpu_baseline leg).

The reference does not vendor the VAE: it calls diffusers' ``AutoencoderKL`` (run_videop2p.py:107-110,
495-537; pipeline_tuneavideo.py:239-256), and diffusers is not installed here, so this restatement of
the published 0.11.1 module semantics is PARITY UNPINNED against the real library:
  Encoder / Decoder (vae.py), DownEncoderBlock2D / UpDecoderBlock2D / UNetMidBlock2D (unet_2d_blocks.py),
  ResnetBlock2D with temb=None, Downsample2D (pad (0,1,0,1) + 3x3 stride-2 conv), Upsample2D (nearest x2 +
  3x3 conv), AttentionBlock (GroupNorm, one head, q*s . (k*s)^T with s = C^-1/4, softmax, proj, residual),
  GroupNorm eps 1e-6, quant_conv / post_quant_conv, DiagonalGaussian mean = first half of the moments.
"""
from __future__ import annotations

import math
from typing import Dict

import torch
import torch.nn.functional as F

EPS = 1e-6


def _gn(x, sd, p, silu):
    y = F.group_norm(x, 32, sd[p + "weight"], sd[p + "bias"], EPS)
    return F.silu(y) if silu else y


def _conv(x, sd, p, stride=1, padding=None):
    w = sd[p + "weight"]
    pad = w.shape[-1] // 2 if padding is None else padding
    return F.conv2d(x, w, sd[p + "bias"], stride=stride, padding=pad)


def resnet(sd, p, x):
    h = _conv(_gn(x, sd, p + "norm1.", True), sd, p + "conv1.")
    h = _conv(_gn(h, sd, p + "norm2.", True), sd, p + "conv2.")
    sc = _conv(x, sd, p + "conv_shortcut.") if (p + "conv_shortcut.weight") in sd else x
    return sc + h


def attention(sd, p, x):
    N, C, H, W = x.shape
    h = _gn(x, sd, p + "group_norm.", False).reshape(N, C, H * W).transpose(1, 2)
    q = F.linear(h, sd[p + "query.weight"], sd[p + "query.bias"])
    k = F.linear(h, sd[p + "key.weight"], sd[p + "key.bias"])
    v = F.linear(h, sd[p + "value.weight"], sd[p + "value.bias"])
    s = 1 / math.sqrt(math.sqrt(C))
    probs = torch.softmax(torch.bmm(q * s, (k * s).transpose(1, 2)), dim=-1)
    out = F.linear(torch.bmm(probs, v), sd[p + "proj_attn.weight"], sd[p + "proj_attn.bias"])
    return out.transpose(1, 2).reshape(N, C, H, W) + x


def mid(sd, p, x):
    x = resnet(sd, p + "resnets.0.", x)
    x = attention(sd, p + "attentions.0.", x)
    return resnet(sd, p + "resnets.1.", x)


def _n_blocks(sd, prefix):
    return 1 + max(int(k[len(prefix):].split(".")[0]) for k in sd if k.startswith(prefix))


def encode_mean(sd: Dict[str, torch.Tensor], images: torch.Tensor) -> torch.Tensor:
    sd = {k: v.float().cpu() for k, v in sd.items()}
    x = _conv(images.float(), sd, "encoder.conv_in.")
    for i in range(_n_blocks(sd, "encoder.down_blocks.")):
        p = f"encoder.down_blocks.{i}."
        for j in range(_n_blocks(sd, p + "resnets.")):
            x = resnet(sd, p + f"resnets.{j}.", x)
        if (p + "downsamplers.0.conv.weight") in sd:
            x = _conv(F.pad(x, (0, 1, 0, 1)), sd, p + "downsamplers.0.conv.", stride=2, padding=0)
    x = mid(sd, "encoder.mid_block.", x)
    x = _conv(_gn(x, sd, "encoder.conv_norm_out.", True), sd, "encoder.conv_out.")
    moments = _conv(x, sd, "quant_conv.")
    return moments[:, :moments.shape[1] // 2]


def decode(sd: Dict[str, torch.Tensor], z: torch.Tensor) -> torch.Tensor:
    sd = {k: v.float().cpu() for k, v in sd.items()}
    x = _conv(_conv(z.float(), sd, "post_quant_conv."), sd, "decoder.conv_in.")
    x = mid(sd, "decoder.mid_block.", x)
    for i in range(_n_blocks(sd, "decoder.up_blocks.")):
        p = f"decoder.up_blocks.{i}."
        for j in range(_n_blocks(sd, p + "resnets.")):
            x = resnet(sd, p + f"resnets.{j}.", x)
        if (p + "upsamplers.0.conv.weight") in sd:
            x = _conv(F.interpolate(x, scale_factor=2.0, mode="nearest"), sd, p + "upsamplers.0.conv.")
    return _conv(_gn(x, sd, "decoder.conv_norm_out.", True), sd, "decoder.conv_out.")
