"""The VAE around the edit: diffusers-0.11.1 ``AutoencoderKL`` (SD-1.5 config)
on the MI355X, frame-parallel.

Reference call sites: ``TuneAVideoPipeline.decode_latents`` (pipeline_tuneavideo.py:239-256: 1/0.18215
scaling, '(b f)' batches of 4 frames, ``(x / 2 + 0.5).clamp(0, 1)``), ``NullInversion.latent2image_video``
/ ``image2latent_video`` (run_videop2p.py:505-537: the posterior mean times 0.18215) and
``AutoencoderKL.from_pretrained(..., subfolder="vae")`` (run_videop2p.py:107-110).  The module tree and
state-dict keys are diffusers 0.11.1's, so an SD-1.5 ``vae/diffusion_pytorch_model.bin`` loads as is.

Every frame is decoded / encoded independently (the VAE is 2-D), so a frame-sharded edit decodes its
own frames with no collective.  On the GPU:
* GroupNorm (+ SiLU) -- K7 (``ops.group_norm``, per-image statistics: frames = 1), channels-last;
* convolutions -- MIOpen (channels-last bf16/fp32; K10 needs Cout % 160 and the VAE's 128/256/512
  channels do not qualify);
* the mid-block single-head attention over H*W tokens (d = 512) -- hipBLASLt batched GEMMs with
  an fp32 softmax, as diffusers' AttentionBlock computes it (scores in the activation dtype,
  softmax upcast to fp32).
There is no CPU path: the modules raise on CPU tensors through the K7 wrapper.
"""
from __future__ import annotations

import math
from typing import List, Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import frame_parallel, ops

SCALING = 0.18215      # pipeline_tuneavideo.py:241, run_videop2p.py:496, 533


def _gn(norm: nn.GroupNorm, x: torch.Tensor, silu: bool) -> torch.Tensor:
    """GroupNorm of a channels-last (N, C, H, W) image batch (+ SiLU) on K7."""
    if not x.is_contiguous(memory_format=torch.channels_last):
        x = x.contiguous(memory_format=torch.channels_last)
    return ops.group_norm(x, norm.num_groups, norm.weight, norm.bias, norm.eps, 1, silu=silu)


def _conv(conv: nn.Conv2d, x: torch.Tensor) -> torch.Tensor:
    y = conv(x)
    return y if y.is_contiguous(memory_format=torch.channels_last) else y.contiguous(memory_format=torch.channels_last)


class ResnetBlock2D(nn.Module):
    """diffusers 0.11.1 ResnetBlock2D without time embedding (VAE: temb_channels=None, eps 1e-6)."""

    def __init__(self, in_channels: int, out_channels: int, groups: int = 32, eps: float = 1e-6):
        super().__init__()
        self.norm1 = nn.GroupNorm(groups, in_channels, eps=eps, affine=True)
        self.conv1 = nn.Conv2d(in_channels, out_channels, 3, padding=1)
        self.norm2 = nn.GroupNorm(groups, out_channels, eps=eps, affine=True)
        self.dropout = nn.Dropout(0.0)
        self.conv2 = nn.Conv2d(out_channels, out_channels, 3, padding=1)
        self.conv_shortcut = nn.Conv2d(in_channels, out_channels, 1) if in_channels != out_channels else None

    def forward(self, x):
        h = _conv(self.conv1, _gn(self.norm1, x, True))
        h = _conv(self.conv2, self.dropout(_gn(self.norm2, h, True)))
        sc = x if self.conv_shortcut is None else _conv(self.conv_shortcut, x)
        return sc + h


class AttentionBlock(nn.Module):
    """diffusers 0.11.1 AttentionBlock (VAE mid block: one head over all H*W positions, d = C)."""

    def __init__(self, channels: int, groups: int = 32, eps: float = 1e-6):
        super().__init__()
        self.channels = channels
        self.num_heads = 1
        self.group_norm = nn.GroupNorm(groups, channels, eps=eps, affine=True)
        self.query = nn.Linear(channels, channels)
        self.key = nn.Linear(channels, channels)
        self.value = nn.Linear(channels, channels)
        self.proj_attn = nn.Linear(channels, channels)

    def forward(self, x):
        N, C, H, W = x.shape
        h = _gn(self.group_norm, x, False).permute(0, 2, 3, 1).reshape(N, H * W, C)   # channels-last: no copy
        scale = 1 / math.sqrt(math.sqrt(C / self.num_heads))
        q = F.linear(h, self.query.weight, self.query.bias)
        k = F.linear(h, self.key.weight, self.key.bias)
        v = F.linear(h, self.value.weight, self.value.bias)
        scores = torch.baddbmm(torch.empty(N, H * W, H * W, dtype=q.dtype, device=q.device), q * scale,
                               k.transpose(-1, -2) * scale, beta=0, alpha=1)
        probs = torch.softmax(scores.float(), dim=-1).to(scores.dtype)
        out = F.linear(torch.bmm(probs, v), self.proj_attn.weight, self.proj_attn.bias)
        out = out.reshape(N, H, W, C).permute(0, 3, 1, 2)
        return out + x


class Downsample2D(nn.Module):
    def __init__(self, channels: int):
        super().__init__()
        self.conv = nn.Conv2d(channels, channels, 3, stride=2, padding=0)

    def forward(self, x):
        return _conv(self.conv, F.pad(x, (0, 1, 0, 1), mode="constant", value=0.0))


class Upsample2D(nn.Module):
    def __init__(self, channels: int):
        super().__init__()
        self.conv = nn.Conv2d(channels, channels, 3, padding=1)

    def forward(self, x):
        dtype = x.dtype
        y = F.interpolate(x.float() if dtype == torch.bfloat16 else x, scale_factor=2.0, mode="nearest").to(dtype)
        return _conv(self.conv, y.contiguous(memory_format=torch.channels_last))


class DownEncoderBlock2D(nn.Module):
    def __init__(self, cin: int, cout: int, layers: int, add_downsample: bool):
        super().__init__()
        self.resnets = nn.ModuleList([ResnetBlock2D(cin if i == 0 else cout, cout) for i in range(layers)])
        self.downsamplers = nn.ModuleList([Downsample2D(cout)]) if add_downsample else None

    def forward(self, x):
        for r in self.resnets:
            x = r(x)
        if self.downsamplers is not None:
            x = self.downsamplers[0](x)
        return x


class UpDecoderBlock2D(nn.Module):
    def __init__(self, cin: int, cout: int, layers: int, add_upsample: bool):
        super().__init__()
        self.resnets = nn.ModuleList([ResnetBlock2D(cin if i == 0 else cout, cout) for i in range(layers)])
        self.upsamplers = nn.ModuleList([Upsample2D(cout)]) if add_upsample else None

    def forward(self, x):
        for r in self.resnets:
            x = r(x)
        if self.upsamplers is not None:
            x = self.upsamplers[0](x)
        return x


class UNetMidBlock2D(nn.Module):
    def __init__(self, channels: int):
        super().__init__()
        self.resnets = nn.ModuleList([ResnetBlock2D(channels, channels), ResnetBlock2D(channels, channels)])
        self.attentions = nn.ModuleList([AttentionBlock(channels)])

    def forward(self, x):
        x = self.resnets[0](x)
        for a, r in zip(self.attentions, self.resnets[1:]):
            x = r(a(x))
        return x


class Encoder(nn.Module):
    def __init__(self, in_channels=3, out_channels=4, block_out_channels=(128, 256, 512, 512), layers=2):
        super().__init__()
        self.conv_in = nn.Conv2d(in_channels, block_out_channels[0], 3, padding=1)
        self.down_blocks = nn.ModuleList()
        cout = block_out_channels[0]
        for i, c in enumerate(block_out_channels):
            cin, cout = cout, c
            self.down_blocks.append(DownEncoderBlock2D(cin, cout, layers, i < len(block_out_channels) - 1))
        self.mid_block = UNetMidBlock2D(block_out_channels[-1])
        self.conv_norm_out = nn.GroupNorm(32, block_out_channels[-1], eps=1e-6)
        self.conv_act = nn.SiLU()
        self.conv_out = nn.Conv2d(block_out_channels[-1], 2 * out_channels, 3, padding=1)

    def forward(self, x):
        x = _conv(self.conv_in, x)
        for blk in self.down_blocks:
            x = blk(x)
        x = self.mid_block(x)
        return _conv(self.conv_out, _gn(self.conv_norm_out, x, True))


class Decoder(nn.Module):
    def __init__(self, in_channels=4, out_channels=3, block_out_channels=(128, 256, 512, 512), layers=2):
        super().__init__()
        self.conv_in = nn.Conv2d(in_channels, block_out_channels[-1], 3, padding=1)
        self.mid_block = UNetMidBlock2D(block_out_channels[-1])
        rev = list(reversed(block_out_channels))
        self.up_blocks = nn.ModuleList()
        cout = rev[0]
        for i, c in enumerate(rev):
            prev, cout = cout, c
            self.up_blocks.append(UpDecoderBlock2D(prev, cout, layers + 1, i < len(rev) - 1))
        self.conv_norm_out = nn.GroupNorm(32, block_out_channels[0], eps=1e-6)
        self.conv_act = nn.SiLU()
        self.conv_out = nn.Conv2d(block_out_channels[0], out_channels, 3, padding=1)

    def forward(self, z):
        x = _conv(self.conv_in, z)
        x = self.mid_block(x)
        for blk in self.up_blocks:
            x = blk(x)
        return _conv(self.conv_out, _gn(self.conv_norm_out, x, True))


class AutoencoderKL(nn.Module):
    """diffusers 0.11.1 AutoencoderKL with the SD-1.5 VAE config (latent 4 channels, 8x down)."""

    def __init__(self, in_channels=3, out_channels=3, latent_channels=4, block_out_channels=(128, 256, 512, 512),
                 layers_per_block=2):
        super().__init__()
        self.encoder = Encoder(in_channels, latent_channels, block_out_channels, layers_per_block)
        self.decoder = Decoder(latent_channels, out_channels, block_out_channels, layers_per_block)
        self.quant_conv = nn.Conv2d(2 * latent_channels, 2 * latent_channels, 1)
        self.post_quant_conv = nn.Conv2d(latent_channels, latent_channels, 1)
        self.latent_channels = latent_channels

    @property
    def dtype(self):
        return self.quant_conv.weight.dtype

    def _in(self, x):
        return x.to(self.dtype).contiguous(memory_format=torch.channels_last)

    def encode_mean(self, images: torch.Tensor) -> torch.Tensor:
        """(N, 3, H, W) in [-1, 1] -> the posterior mean (N, 4, H/8, W/8) (``latent_dist.mean``)."""
        moments = _conv(self.quant_conv, self.encoder(self._in(images)))
        return moments[:, :self.latent_channels]

    def decode(self, z: torch.Tensor) -> torch.Tensor:
        """(N, 4, h, w) latents (already divided by the scaling factor) -> (N, 3, 8h, 8w) ``.sample``."""
        return self.decoder(_conv(self.post_quant_conv, self._in(z)))


def init_vae_random_(vae: nn.Module, seed: int = 0) -> nn.Module:
    """Synthetic VAE weights (no checkpoint offline): conv/linear ~ N(0, 1/fan_in) so activations
    stay O(1) through the ~40 layers, biases 0, norms (1, 0)."""
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for m in vae.modules():
            if isinstance(m, (nn.Linear, nn.Conv2d)):
                fan_in = m.weight[0].numel()
                m.weight.copy_(torch.randn(m.weight.shape, generator=g) / math.sqrt(fan_in))
                if m.bias is not None:
                    m.bias.zero_()
            elif isinstance(m, nn.GroupNorm):
                m.weight.fill_(1.0)
                m.bias.zero_()
    return vae


@torch.no_grad()
def decode_latents(vae: AutoencoderKL, latents: torch.Tensor, chunk: int = 4) -> torch.Tensor:
    """TuneAVideoPipeline.decode_latents (pipeline_tuneavideo.py:239-256) on the GPU: (b, 4, f, h, w)
    latents -> (b, 3, f, 8h, 8w) video in [0, 1] (fp32, on the device).  Frames are decoded in
    '(b f)' batches of ``chunk`` (the reference's bs = 4).  As in the reference loop
    (``range(max(n // bs, 1))``), a trailing partial batch is never decoded when n > bs is not a
    multiple of bs, so the reference's ``rearrange(..., f=video_length)`` raises; this raises
    ``ValueError`` in the same case (judged on the global frame count under frame sharding, where
    each rank decodes all of its own frames)."""
    b, c, f, h, w = latents.shape
    sh = frame_parallel.active()
    n_global = b * f * (sh.world if sh is not None else 1)
    if n_global > chunk and n_global % chunk:
        raise ValueError(f"decode_latents: {n_global} frames are not a multiple of the decode batch {chunk} "
                         f"(the reference drops the trailing {n_global % chunk} and its rearrange fails)")
    x = (1 / SCALING) * latents
    x = x.permute(0, 2, 1, 3, 4).reshape(b * f, c, h, w)
    n = x.shape[0]
    outs = []
    for i in range(0, n, chunk):
        v = vae.decode(x[i:min(i + chunk, n)])
        outs.append((v.float() / 2 + 0.5).clamp(0, 1))
    video = torch.cat(outs)
    return video.reshape(b, f, *video.shape[1:]).permute(0, 2, 1, 3, 4)


@torch.no_grad()
def encode_video(vae: AutoencoderKL, frames: torch.Tensor) -> torch.Tensor:
    """NullInversion.image2latent_video (run_videop2p.py:529-537) on the GPU: (f, H, W, 3) uint8
    frames -> (1, 4, f, H/8, W/8) fp32 latents = posterior mean * 0.18215."""
    img = frames.to(torch.float32) / 127.5 - 1
    img = img.permute(0, 3, 1, 2)
    lat = vae.encode_mean(img).float()
    f = lat.shape[0]
    return (lat.reshape(1, f, *lat.shape[1:]).permute(0, 2, 1, 3, 4) * SCALING).contiguous()


@torch.no_grad()
def latent2image_video(vae: AutoencoderKL, latents: torch.Tensor) -> torch.Tensor:
    """NullInversion.latent2image_video (run_videop2p.py:505-513): latents[0] of (b, 4, f, h, w) ->
    (f, 8h, 8w, 3) uint8 frames."""
    x = (1 / SCALING) * latents[0].permute(1, 0, 2, 3)
    image = (vae.decode(x).float() / 2 + 0.5).clamp(0, 1)
    return (image.permute(0, 2, 3, 1) * 255).to(torch.uint8)


def gather_frames(video: torch.Tensor, dim: int = 2) -> torch.Tensor:
    """All ranks' decoded frames of a frame-sharded edit, concatenated along ``dim`` (identity when
    frames are not sharded)."""
    sh = frame_parallel.active()
    return video if sh is None else sh.gather(video, dim)
