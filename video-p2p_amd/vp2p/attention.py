"""Attention modules of the video UNet and the drop-in ``register_attention_control``.

``CrossAttention`` exposes the diffusers-0.11.1 attribute set the reference hook relies on
(to_q / to_k / to_v / to_out[0], heads, scale, reshape_heads_to_batch_dim,
reshape_batch_dim_to_heads; ptp_utils.py:189-208), so ``register_attention_control`` patches our
modules and the reference's tuneavideo modules alike.  Its patched forward runs the hooked math
of ptp_utils.py:196-221 on the HIP kernels:

* cross  (attn2)    -> K2  ``vp2p_cross_attn_p2p_fwd``   (edit + LocalBlend reduction fused)
* self   (attn_temp)-> K3  ``vp2p_temporal_attn_p2p_fwd`` (self-replace fused)
* FrameAttention (attn1, never hooked in the reference: its class name differs,
  ptp_utils.py:237) -> K1 ``vp2p_frame_attn_fwd``

Projections go through ``ops.linear`` (K10's GEMM core where the in-tree table measured it faster,
hipBLASLt elsewhere); K/V of attn1 are projected for frame 0 only,
K/V of attn2 once per batch row instead of once per frame, and attn_temp's q/k/v come from one GEMM
against the concatenated weights -- all bit-identical to the reference's per-row projections.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import autograd, frame_parallel, ops
from .controllers import LayerCall


def _cat_weight(module: nn.Module, names, cache_attr: str) -> torch.Tensor:
    ws = [getattr(module, n).weight for n in names]
    key = ops.version_key(*ws)
    hit = getattr(module, cache_attr, None)
    if hit is not None and key is not None and hit[0] == key:
        return hit[1]
    cat = torch.cat([w.detach() for w in ws], 0).contiguous()
    if key is None:
        return cat
    # the entry holds the weights themselves: a replaced parameter cannot reuse their memory (and so
    # their key) while the entry lives
    object.__setattr__(module, cache_attr, (key, cat, tuple(ws)))
    return cat


class CrossAttention(nn.Module):
    """diffusers 0.11.1 ``CrossAttention`` parameter layout (bias-free q/k/v, to_out = [Linear,
    Dropout]); forward = plain (un-hooked) attention on the HIP kernels."""

    def __init__(self, query_dim: int, cross_attention_dim: Optional[int] = None, heads: int = 8,
                 dim_head: int = 64, dropout: float = 0.0, bias: bool = False,
                 upcast_attention: bool = False):
        super().__init__()
        inner = heads * dim_head
        ctx = cross_attention_dim if cross_attention_dim is not None else query_dim
        self.heads = heads
        self.scale = dim_head ** -0.5
        self.upcast_attention = upcast_attention
        self.to_q = nn.Linear(query_dim, inner, bias=bias)
        self.to_k = nn.Linear(ctx, inner, bias=bias)
        self.to_v = nn.Linear(ctx, inner, bias=bias)
        self.to_out = nn.ModuleList([nn.Linear(inner, query_dim), nn.Dropout(dropout)])

    def reshape_heads_to_batch_dim(self, t):
        b, n, dim = t.shape
        h = self.heads
        return t.reshape(b, n, h, dim // h).permute(0, 2, 1, 3).reshape(b * h, n, dim // h)

    def reshape_batch_dim_to_heads(self, t):
        bh, n, d = t.shape
        h = self.heads
        return t.reshape(bh // h, h, n, d).permute(0, 2, 1, 3).reshape(bh // h, n, h * d)

    def forward(self, hidden_states, encoder_hidden_states=None, attention_mask=None, video_length=None,
                temporal_layout=None, residual=None):
        return hooked_attention(self, None, "none", hidden_states, encoder_hidden_states, attention_mask,
                                video_length, temporal_layout, residual)


class FrameAttention(CrossAttention):
    """Sparse-causal frame attention with first-frame K/V (attention.py:273-329) on K1."""

    def forward(self, hidden_states, encoder_hidden_states=None, attention_mask=None, video_length=None,
                residual=None):
        """``residual``: return residual + attn(x) (the block's add, attention.py:247-252), the add in
        the output projection's epilogue (inference only)."""
        if attention_mask is not None:
            raise NotImplementedError("FrameAttention: attention_mask (never passed by the UNet)")
        if encoder_hidden_states is not None:
            raise NotImplementedError("FrameAttention: only_cross_attention")
        x = hidden_states
        f = video_length
        B = x.shape[0] // f
        shard = frame_parallel.active()
        pending = None
        differentiated = autograd.needs_grad(x, self.to_q.weight, self.to_q.bias)
        if shard is not None and shard.world > 1 and not differentiated:
            # frames are sharded: the rank owning frame 0 broadcasts frame 0's NORMED hidden state
            # (C per token, half the bytes of its K|V) and every rank projects K|V itself.  The
            # broadcast is issued before this rank's Q projection so the two overlap (collective
            # stream vs compute stream).
            x0 = (x.view(B, f, *x.shape[1:])[:, 0].contiguous() if shard.rank == 0
                  else torch.empty(B, *x.shape[1:], device=x.device, dtype=x.dtype))
            pending = (x0, shard.broadcast_async(x0))
        if differentiated:
            q = ops.linear(x, self.to_q.weight, self.to_q.bias)
            prescaled = False
        else:
            # the softmax scale (times log2 e) rides in the projection GEMM's alpha: one rounding of
            # q' = c * (x W^T + b), and K1 runs its folded-max form (frame_attn.hip)
            q = ops.linear(x, self.to_q.weight, self.to_q.bias,
                           alpha=ops.frame_query_scale(self.to_q.weight.shape[0] // self.heads, self.scale))
            prescaled = True
        C = q.shape[-1]
        if not prescaled:
            x0 = x.view(B, f, *x.shape[1:])[:, 0]
            if shard is not None and shard.world > 1:
                # frames sharded under autograd (null-text): rank 0's frame-0 hidden state, with the
                # adjoint (its gradient summed over the ranks that projected K|V from it)
                x0 = frame_parallel.frame0_hidden(shard, x0)
            kv = ops.linear(x0, _cat_weight(self, ("to_k", "to_v"), "_wkv"),
                            None if self.to_k.bias is None else torch.cat([self.to_k.bias, self.to_v.bias]))
            out = autograd.SharedKVAttention.apply(q, kv, f, self.heads, self.scale)
            y = self.to_out[1](_linear_out(self.to_out[0], out))
            return y if residual is None else y + residual
        wkv = _cat_weight(self, ("to_k", "to_v"), "_wkv")
        bkv = None if self.to_k.bias is None else torch.cat([self.to_k.bias, self.to_v.bias])
        if pending is not None:
            x0, work = pending
            work.wait()
        else:
            if shard is not None and shard.world > 1:
                raise RuntimeError("frame-sharded FrameAttention reached the inference path without "
                                   "the frame-0 broadcast")
            x0 = x.view(B, f, *x.shape[1:])[:, 0]
        kv = ops.linear(x0, wkv, bkv)
        out = ops.frame_attention(q, kv[..., :C], kv[..., C:], f, self.heads, scale=self.scale,
                                  q_prescaled=True)
        if residual is not None:
            return _linear_out_add(self.to_out[0], out, residual)
        return self.to_out[1](_linear_out(self.to_out[0], out))




def _context_kv(module, ctx: torch.Tensor, heads: int):
    """K and V of the (B, 77, Cctx) text context (one GEMM against [Wk; Wv]) and K2's fragment-order
    layout of them.  The context is the same tensor at every denoising step of an edit (the UNet hands
    out one converted copy while its input is unchanged), so both are kept until the context or the
    weights change: the reference recomputes to_k / to_v(context) per step (ptp_utils.py:204-205) with
    identical results.  A changed context (null-text: a new unconditional embedding per step; an
    in-place write bumps ``_version``) recomputes them.  The cache holds the context tensor itself, so
    its memory cannot be recycled under an equal key."""
    wkv = _cat_weight(module, ("to_k", "to_v"), "_wkv")
    # the parameters themselves (storage and version), not the concatenated copy, whose memory is
    # recycled when the weights change
    pkey = ops.version_key(*(p for m in (module.to_k, module.to_v) for p in (m.weight, m.bias) if p is not None))
    ckey = ops.version_key(ctx)
    key = (ckey, tuple(ctx.shape), tuple(ctx.stride()), pkey, heads)
    # a HIP graph records the projection itself; inference tensors have no version counter to key on
    capturing = torch.cuda.is_current_stream_capturing() or ckey is None or pkey is None
    hit = getattr(module, "_ctx_kv", None)
    if hit is not None and hit[0] == key and not capturing:
        return hit[2], hit[3], hit[4]
    kv = ops.linear(ctx, wkv, None if module.to_k.bias is None else torch.cat([module.to_k.bias, module.to_v.bias]))
    Ck = module.to_k.weight.shape[0]
    k, v = kv[..., :Ck], kv[..., Ck:]
    ws = ops.cross_kv_prep(k, v, heads)
    if not capturing:     # held: ctx and the parameters (their memory cannot be recycled under the key)
        params = tuple(p for m in (module.to_k, module.to_v) for p in (m.weight, m.bias) if p is not None)
        object.__setattr__(module, "_ctx_kv", (key, ctx, k, v, ws, params))
    return k, v, ws


def _batch_frames(x, controller, video_length):
    P = getattr(controller, "batch_size", 0) or 0
    if video_length:
        return x.shape[0] // video_length, video_length, P
    if P and x.shape[0] % (2 * P) == 0:
        return 2 * P, x.shape[0] // (2 * P), P
    return x.shape[0], 1, 0


def _p2p_rows(B: int, P: int):
    """(prompts, cond_only) for the attention kernels: the batch is [uncond x P, cond x P]
    (prompts = P) -- or, on a rank of a CFG-split edit (frame_parallel.EditLayout), only the
    unconditional rows (plain attention: prompts = 0) or only the conditional rows (cond_only)."""
    lay = frame_parallel.active_layout()
    if lay is not None and lay.cfg_split:
        return (P, True) if (lay.half == 1 and P and B == P) else (0, False)
    return (P if (P and B == 2 * P) else 0), False


def hooked_attention(module, controller, place, x, context=None, attention_mask=None, video_length=None,
                     temporal_layout=None, residual=None):
    """The patched forward (ptp_utils.py:196-221) for ``controller`` on the HIP kernels."""
    if attention_mask is not None:
        raise NotImplementedError("attention_mask is not supported on the fused path "
                                  "(the reference UNet never passes one, pipeline_tuneavideo.py:406)")
    is_cross = context is not None
    fused = controller is None or getattr(controller, "fused", False)
    h = module.heads
    to_out = module.to_out[0] if isinstance(module.to_out, nn.ModuleList) else module.to_out
    dev = x.device

    plain = controller is None or isinstance(controller, DummyController)
    if is_cross:
        B, f, P = _batch_frames(x, controller, video_length)
        N = x.shape[1]
        P, cond_only = _p2p_rows(B, P)
        # the context is repeated per frame (attention.py:95); project it once per batch row
        ctx = context if context.shape[0] == B else context.reshape(B, f, *context.shape[1:])[:, 0]
        if autograd.needs_grad(x, ctx):
            # differentiated (null-text optimisation): only the uncontrolled hook is ever traced there
            if not plain:
                raise NotImplementedError("backward through a P2P-controlled attention layer")
            q = ops.linear(x, module.to_q.weight, module.to_q.bias)
            kv = ops.linear(ctx, _cat_weight(module, ("to_k", "to_v"), "_wkv"),
                            None if module.to_k.bias is None else torch.cat([module.to_k.bias, module.to_v.bias]))
            y = _linear_out(to_out, autograd.SharedKVAttention.apply(q, kv, f, h, module.scale))
            return y if residual is None else y + residual
        q = ops.linear(x, module.to_q.weight, module.to_q.bias)
        k, v, kv_ws = _context_kv(module, ctx, h)
        call = controller.fused_begin(True, place, N, f) if (controller is not None and fused) else LayerCall()
        call.cond_only = cond_only
        probs = None
        if call.store or not fused:
            probs = torch.empty(B * f * h, N, k.shape[1], device=dev, dtype=torch.float32)
        plan = None
        lb = None
        if fused and controller is not None and P and (call.edit or call.lb_acc):
            plan = controller.plan(dev)
            if call.lb_acc:
                lb = controller.lb_buffer(f, dev)
        out = ops.cross_attention_p2p(q, k, v, f, h, plan=plan, step=call.step, edit=call.edit, lb_acc=lb,
                                      probs_out=probs, prompts=P, scale=module.scale, cond_only=cond_only,
                                      kv_ws=kv_ws)
        if not fused:
            attn = controller(probs, True, place)
            out = _pv(module, attn, v.contiguous(), B, f)
        elif controller is not None:
            controller.fused_end(True, place, call, probs)
        if residual is not None:
            return _linear_out_add(to_out, out, residual)
        return _linear_out(to_out, out)

    # self attention on the hooked path = temporal attention (attn_temp)
    C = module.to_q.weight.shape[0]
    w = _cat_weight(module, ("to_q", "to_k", "to_v"), "_wqkv")
    bias = None
    if module.to_q.bias is not None:
        bias = torch.cat([module.to_q.bias, module.to_k.bias, module.to_v.bias])
    if autograd.needs_grad(x, w, bias):
        if not plain or temporal_layout != "bf":
            raise NotImplementedError("backward through a P2P-controlled or '(b d) f c' temporal attention")
        sh = frame_parallel.active()
        if sh is not None and sh.world > 1:
            # frames sharded under autograd: the all-to-all frames <-> tokens (of the normed hidden
            # state: C per token, the projection runs on the token slice) and its adjoint
            Bq = x.shape[0] // video_length
            qkv = ops.linear(frame_parallel.to_tokens(sh, x, Bq), w, bias)
            out = autograd.TemporalAttention.apply(qkv, video_length * sh.world, h, module.scale)
            return _linear_out(to_out, frame_parallel.to_frames(sh, out, Bq))
        return _linear_out(to_out, autograd.TemporalAttention.apply(ops.linear(x, w, bias), video_length, h, module.scale))
    shard = frame_parallel.active() if temporal_layout == "bf" else None
    if shard is not None and shard.world <= 1:
        shard = None
    if temporal_layout == "bf":
        f = video_length * (shard.world if shard is not None else 1)
        B = x.shape[0] // video_length
        N = x.shape[1] // (shard.world if shard is not None else 1)   # this rank's token slice
    else:  # the reference's '(b d) f c' tensor
        f = x.shape[1]
        P0 = getattr(controller, "batch_size", 0) or 0
        B = 2 * P0 if (P0 and x.shape[0] % (2 * P0) == 0) else 1
        N = x.shape[0] // B
    P, cond_only = _p2p_rows(B, getattr(controller, "batch_size", 0) or 0)
    call = controller.fused_begin(False, place, f, f) if (controller is not None and fused) else LayerCall()
    call.cond_only = cond_only
    probs = None
    if call.store or not fused:
        probs = torch.empty(B * N * h, f, f, device=dev, dtype=torch.float32)
    replace = bool(call.self_replace) and P > 0

    def kernel(xt):
        """q|k|v projection + K3 (+ the foreign controller) on (B*f, n, C) tokens -> (B*f, n, C)."""
        qkv = ops.linear(xt, w, bias)
        q, k, v = qkv[..., :C], qkv[..., C:2 * C], qkv[..., 2 * C:]
        if temporal_layout == "bf":
            o = ops.temporal_attention_p2p(q, k, v, f, h, prompts=P, self_replace=replace, probs_out=probs,
                                           scale=module.scale, cond_only=cond_only)
        else:
            o = ops.temporal_attention_p2p_bd(q, k, v, B, h, prompts=P, self_replace=replace, probs_out=probs,
                                              scale=module.scale, cond_only=cond_only)
        if not fused:
            attn = controller(probs, False, place)
            o = _pv_temporal(module, attn, v, B, f, qkv.shape[1] if temporal_layout == "bf" else N, temporal_layout == "bf")
        return o

    if shard is not None:
        # one exchange of the normed hidden state per direction, in token pieces that overlap the
        # kernel (one piece when the probabilities are materialised for a controller)
        out = shard.temporal_exchange(x, B, kernel, 1 if probs is not None else _temporal_chunks(x, shard.world))
    else:
        out = kernel(x)
    if fused and controller is not None:
        controller.fused_end(False, place, call, probs)
    return _out_proj(to_out, out, residual)


def _temporal_chunks(x: torch.Tensor, world: int) -> int:
    """Token pieces of the sharded attn_temp exchange: 4 when each piece still moves >= 1 MiB per
    rank, else 1 (small messages are latency-bound; splitting them only adds launches)."""
    per_rank = x.numel() * x.element_size() // max(world, 1)
    return 4 if per_rank >= 4 << 20 and (x.shape[1] // world) % 4 == 0 else 1


def _plain_linear(m) -> bool:
    """A bare nn.Linear with no forward hooks: only then may its weights be used directly (a subclass
    such as a LoRA-compatible Linear, or a hooked module, is called as a module)."""
    return type(m) is nn.Linear and not (m._forward_hooks or m._forward_pre_hooks)


def _linear_out(to_out, out):
    """``to_out(out)`` through ``ops.linear`` (K10's GEMM core for the K = 320 projections of the 64x64
    latents, hipBLASLt elsewhere; under autograd with frozen weights the same dispatch forward and
    backward); any other module is called as is."""
    if _plain_linear(to_out):
        return ops.linear(out, to_out.weight, to_out.bias)
    return to_out(out)


def _linear_out_add(to_out, out, residual):
    """residual + to_out(out) (the block's residual add, attention.py:247-262) at inference: the add
    in K10's epilogue where the projection runs on K10 (``ops.linear_add``), the two roundings of
    the reference (projection, then sum) either way."""
    if _plain_linear(to_out) and not torch.is_grad_enabled() and out.is_contiguous():
        return ops.linear_add(out, to_out.weight, to_out.bias, residual)
    return to_out(out) + residual


def _out_proj(to_out, out, residual):
    """``to_out(out)``, plus ``residual`` when the caller passes the block's residual
    (``attn_temp(norm_temp(x)) + x``, attention.py:268).  At inference the add runs in the epilogue
    of K10's GEMM core when the in-tree kernel-choice table says it is faster for the shape than
    hipBLASLt + a separate add (``ops.CONV.pick``, the same per-shape choice as the proj_out fusion)."""
    if residual is None:
        return to_out(out)
    if torch.is_grad_enabled() or not _plain_linear(to_out) or not out.is_contiguous() \
            or residual.shape[:-1] != out.shape[:-1] or residual.dtype != out.dtype:
        return to_out(out) + residual
    res = residual.contiguous()

    def fused():
        return ops.linear_residual(out, to_out.weight, to_out.bias, res)

    def lib():
        return to_out(out) + res

    key = ("to_out_res", tuple(out.shape), tuple(to_out.weight.shape))
    ok = ops.linear_residual_supported(out, to_out.weight, res)
    return fused() if ops.CONV.pick(key, ok, fused, lib) else lib()


def _pv(module, attn, v, B, f):
    """attn @ v for a foreign controller's edited maps: (B*f*h, N, M) x (B, M, C)."""
    h = module.heads
    vb = module.reshape_heads_to_batch_dim(v.repeat_interleave(f, 0)).to(attn.dtype)
    out = torch.bmm(attn, vb)
    return module.reshape_batch_dim_to_heads(out).to(v.dtype)


def _pv_temporal(module, attn, v, B, f, N, bf_layout):
    h = module.heads
    C = v.shape[-1]
    if bf_layout:
        vv = v.reshape(B, f, N, C).permute(0, 2, 1, 3).reshape(B * N, f, C)
    else:
        vv = v
    out = torch.bmm(attn, module.reshape_heads_to_batch_dim(vv).to(attn.dtype))
    out = module.reshape_batch_dim_to_heads(out).to(v.dtype)
    if bf_layout:
        out = out.reshape(B, N, f, C).permute(0, 2, 1, 3).reshape(B * f, N, C)
    return out


class DummyController:
    """ptp_utils.py:225-234."""

    fused = True

    def __call__(self, *args):
        return args[0]

    def __init__(self):
        self.num_att_layers = 0

    def fused_begin(self, *a):
        return LayerCall()

    def fused_end(self, *a):
        return None


def _frame_forward(net):
    """Forward for a foreign module whose class is named ``FrameAttention`` (the reference's attn1,
    tuneavideo/models/attention.py:273-329, signature :274): the same K1 path as ours
    (``FrameAttention.forward``), on the module's own to_q / to_k / to_v / to_out, heads and scale.
    The reference's xformers / sliced-attention switches select among equal maths there and are
    ignored here; the options its UNet never uses raise, as ours do."""
    def forward(hidden_states, encoder_hidden_states=None, attention_mask=None, video_length=None,
                residual=None):
        if getattr(net, "group_norm", None) is not None or getattr(net, "added_kv_proj_dim", None) is not None:
            raise NotImplementedError("FrameAttention: group_norm / added_kv_proj_dim")
        if video_length is None:
            raise ValueError("FrameAttention needs video_length (attention.py:293)")
        if hidden_states.dtype not in (torch.float32, torch.bfloat16):
            # K1 computes in fp32 or bf16; an fp16 reference UNet (run_videop2p.py:93 mixed
            # precision) is not supported
            raise NotImplementedError(f"FrameAttention on the HIP kernels: dtype {hidden_states.dtype} "
                                      "(supported: torch.float32, torch.bfloat16)")
        return FrameAttention.forward(net, hidden_states, encoder_hidden_states, attention_mask,
                                      video_length, residual)
    return forward


def register_attention_control(model, controller):
    """ptp_utils.py:188-255: patch every module whose class is named ``CrossAttention`` under the
    UNet's down*/up*/mid* children; set ``controller.num_att_layers``.

    Beyond the reference: modules whose class is named ``FrameAttention`` (attn1, which the
    reference's hook never reaches: its class name differs, ptp_utils.py:237) are routed to K1
    too, so the reference's own UNet runs every attention on the kernels.  They are not hooked by
    the controller (the reference edits only attn2 / attn_temp) and are not counted in
    ``num_att_layers`` (32 for SD-1.5, as the reference counts)."""
    ctrl = DummyController() if controller is None else controller

    def make_forward(net, place):
        def forward(x, encoder_hidden_states=None, attention_mask=None, video_length=None,
                    temporal_layout=None, residual=None):
            return hooked_attention(net, None if controller is None else ctrl, place, x,
                                    encoder_hidden_states, attention_mask, video_length, temporal_layout,
                                    residual)
        return forward

    def walk(net, count, place):
        if net.__class__.__name__ == "CrossAttention":
            net.forward = make_forward(net, place)
            return count + 1
        if net.__class__.__name__ == "FrameAttention":
            if not isinstance(net, FrameAttention):        # ours already runs on K1
                net.forward = _frame_forward(net)
            return count
        for child in net.children():
            count = walk(child, count, place)
        return count

    total = 0
    for name, child in model.unet.named_children():
        if "down" in name:
            total += walk(child, 0, "down")
        elif "up" in name:
            total += walk(child, 0, "up")
        elif "mid" in name:
            total += walk(child, 0, "mid")
    ctrl.num_att_layers = total
    return ctrl
