"""Autograd wrappers of the HIP kernels, for the null-text optimisation.

``NullInversion.null_optimization`` (run_videop2p.py:580-612) back-propagates an MSE on the DDIM
step through the whole UNet to the unconditional text embedding.  Convolutions and projection GEMMs
differentiate through PyTorch (MIOpen / hipBLASLt); every op this package implements as a HIP kernel
gets its backward as a HIP kernel too:

* ``SharedKVAttention``  K1 forward (+ row lse) / K1b backward -- FrameAttention (attention.py:282-322)
  and the plain hooked cross-attention (ptp_utils.py:206-220 under the DummyController)
* ``TemporalAttention``  K3 forward / K3b backward -- plain hooked attn_temp (attention.py:262-268)
* ``GroupNormFn``        K7 / K7b,  ``LayerNormFn`` K8 / K8b,  ``GEGLUFn`` K9 / K9b
* ``FrozenLinear``       a projection with frozen weights: forward through ``ops.linear`` (K10's GEMM
  core or hipBLASLt, per the in-tree table, as at inference), backward dx = dy @ W the same way
* ``FrozenConv``         an InflatedConv3d with frozen weights: forward through the inference dispatch
  (K10 per the in-tree table / MIOpen), backward dx on K10 as a forward convolution (3x3 stride 1:
  dy * the flipped, transposed kernel; 1x1: dy @ W), MIOpen's backward-data elsewhere

Frame-sharded (``frame_parallel``): every cross-frame coupling has a differentiable exchange --
``GroupNormFn`` gathers forward and backward statistics partials, FrameAttention's frame-0 hidden
state and attn_temp's all-to-alls carry their adjoints (``frame_parallel.frame0_hidden`` /
``to_tokens`` / ``to_frames``).

(Round 6: the projections and convolutions of the null-text loop moved from torch autograd --
hipBLASLt / MIOpen forward and backward -- to the two frozen-weight functions above.)

Only input gradients exist: the reference optimises the embedding alone (its Adam holds
``[uncond_embeddings]``, run_videop2p.py:589), so weight gradients are never consumed; asking for
one raises instead of returning a silent zero.
"""
from __future__ import annotations

import torch

from . import ops


def needs_grad(*ts) -> bool:
    return torch.is_grad_enabled() and any(t is not None and t.requires_grad for t in ts)


def _no_weight_grad(ctx, *idx):
    for i in idx:
        if ctx.needs_input_grad[i]:
            raise NotImplementedError("vp2p kernels provide input gradients only (freeze the UNet weights: "
                                      "the null-text optimisation trains the embedding alone)")


class SharedKVAttention(torch.autograd.Function):
    """softmax(scale q k^T) v with the keys/values of batch element b shared by its `frames` frames.
    q: (B*f, N, C); kv: (B, Nk, 2C) = [K | V]."""

    @staticmethod
    def forward(ctx, q, kv, frames: int, heads: int, scale: float):
        q = q.contiguous()
        kv = kv.contiguous()
        C = q.shape[-1]
        B = q.shape[0] // frames
        lse = torch.empty(B, heads, frames * q.shape[1], device=q.device, dtype=torch.float32)
        out = ops.frame_attention(q, kv[..., :C], kv[..., C:], frames, heads, scale=scale, lse=lse)
        ctx.save_for_backward(q, kv, out, lse)
        ctx.cfg = (frames, heads, scale)
        return out

    @staticmethod
    def backward(ctx, dout):
        q, kv, out, lse = ctx.saved_tensors
        frames, heads, scale = ctx.cfg
        C = q.shape[-1]
        dout = dout.contiguous()
        dq = torch.empty_like(q)
        dkv = torch.empty_like(kv)
        ops.frame_attention_bwd(q, kv[..., :C], kv[..., C:], out, dout, lse, frames, heads, scale,
                                dq, dkv[..., :C], dkv[..., C:])
        return dq, dkv, None, None, None


class TemporalAttention(torch.autograd.Function):
    """Plain attention over frames per (b, token, head); qkv: (B*f, N, 3C) = [Q | K | V]."""

    @staticmethod
    def forward(ctx, qkv, frames: int, heads: int, scale: float):
        qkv = qkv.contiguous()
        C = qkv.shape[-1] // 3
        out = ops.temporal_attention_p2p(qkv[..., :C], qkv[..., C:2 * C], qkv[..., 2 * C:], frames, heads,
                                         scale=scale)
        ctx.save_for_backward(qkv)
        ctx.cfg = (frames, heads, scale)
        return out

    @staticmethod
    def backward(ctx, dout):
        (qkv,) = ctx.saved_tensors
        frames, heads, scale = ctx.cfg
        C = qkv.shape[-1] // 3
        dqkv = torch.empty_like(qkv)
        ops.temporal_attention_bwd(qkv[..., :C], qkv[..., C:2 * C], qkv[..., 2 * C:], dout.contiguous(), frames,
                                   heads, scale, dqkv[..., :C], dqkv[..., C:2 * C], dqkv[..., 2 * C:])
        return dqkv, None, None, None


class GroupNormFn(torch.autograd.Function):
    """5-D GroupNorm (+ channel add, + SiLU) of a channels-last '(b f) c h w' tensor.  ``shard``: a
    FrameShard holding the other frames -- the forward all-gathers the statistics partials, the
    backward its (sum dy, sum dy x^) partials, so both passes see the whole clip's statistics."""

    @staticmethod
    def forward(ctx, x, add, weight, bias, groups: int, eps: float, frames: int, silu: bool, shard=None):
        shard = shard if (shard is not None and shard.world > 1) else None
        out, stats = ops.group_norm(x, groups, weight, bias, eps, frames, silu=silu, add=add, return_stats=True,
                                    shard=shard)
        ctx.save_for_backward(x, add, weight, bias, stats[0])
        ctx.cfg = (groups, eps, frames, silu, stats[1], shard)
        return out

    @staticmethod
    def backward(ctx, dy):
        _no_weight_grad(ctx, 1, 2, 3)
        x, add, weight, bias, partials = ctx.saved_tensors
        groups, eps, frames, silu, nsets, shard = ctx.cfg
        dx = ops.group_norm_bwd(x, dy, (partials, nsets), groups, weight, bias, eps, frames, silu=silu, add=add,
                                shard=shard)
        return dx, None, None, None, None, None, None, None, None


class LayerNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, eps: float):
        x = x.contiguous()
        ctx.save_for_backward(x, weight)
        ctx.eps = eps
        return ops.layer_norm(x, weight, bias, eps)

    @staticmethod
    def backward(ctx, dy):
        _no_weight_grad(ctx, 1, 2)
        x, weight = ctx.saved_tensors
        return ops.layer_norm_bwd(x, dy, weight, ctx.eps), None, None, None


class GEGLUFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h):
        h = h.contiguous()
        ctx.save_for_backward(h)
        return ops.geglu(h)

    @staticmethod
    def backward(ctx, dy):
        (h,) = ctx.saved_tensors
        return ops.geglu_bwd(h, dy)


class NullTextLoss(torch.autograd.Function):
    """loss = mse(prev_step(u + g (c - u), t, x), x_prev) of run_videop2p.py:594-599 on K6b; the
    gradient w.r.t. the unconditional noise u comes out of the same pass."""

    @staticmethod
    def forward(ctx, noise_uncond, noise_cond, latents, latents_prev, consts, guidance: float):
        loss, grad = ops.nulltext_loss(noise_uncond.contiguous(), noise_cond.contiguous(), latents.contiguous(),
                                       latents_prev.contiguous(), consts, guidance)
        ctx.save_for_backward(grad)
        return loss

    @staticmethod
    def backward(ctx, dloss):
        (grad,) = ctx.saved_tensors
        return grad * dloss.to(grad.dtype), None, None, None, None, None


def frozen(*ts) -> bool:
    """Weights (and bias) that take no gradient: the frozen-weight functions below apply."""
    return all(t is None or not t.requires_grad for t in ts)


class FrozenLinear(torch.autograd.Function):
    """x @ W^T + b with W, b frozen (the UNet during the null-text optimisation, run_videop2p.py:589
    optimises the embedding alone): the forward is the inference projection (``ops.linear``: K10 or
    hipBLASLt by the in-tree table), the backward dx = dy @ W is ``ops.linear`` on a cached W^T."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        ctx.save_for_backward(weight)
        return ops.linear(x.contiguous(), weight, bias)

    @staticmethod
    def backward(ctx, dy):
        (w,) = ctx.saved_tensors
        return ops.linear(dy.contiguous(), ops.transposed_weight(w)), None, None


class FrozenConv(torch.autograd.Function):
    """An InflatedConv3d (``(b f) c h w`` channels-last) with frozen weights: ``run`` is the module's
    inference convolution (K10 with the fused bias / residual / two-source input, or MIOpen, per the
    in-tree table); the backward gives dx (split into the two sources when the input is
    ``cat([x, x2])``) and d(residual) = dy, the input gradient through ``ops.conv2d_input_grad``."""

    @staticmethod
    def forward(ctx, x, x2, residual, weight, stride, padding, run):
        ctx.save_for_backward(weight)
        ctx.geom = (stride, padding, x.shape[1], None if x2 is None else x2.shape[1],
                    (x.shape[0], x.shape[1] + (0 if x2 is None else x2.shape[1])) + tuple(x.shape[2:]))
        ctx.has_res = residual is not None
        return run()

    @staticmethod
    def backward(ctx, dy):
        (w,) = ctx.saved_tensors
        stride, padding, c1, c2, in_shape = ctx.geom
        dcat = ops.conv2d_input_grad(in_shape, w, dy, stride, padding)
        dx, dx2 = (dcat, None) if c2 is None else (dcat[:, :c1], dcat[:, c1:])
        return dx, dx2, (dy if ctx.has_res else None), None, None, None, None
