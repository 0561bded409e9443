"""Torch-facing wrappers over the C ABI (torch supplies device memory and the stream only).

Every op here launches a HIP kernel from libvp2p_hip.so on ``torch.cuda.current_stream()``;
there is no CPU path.  Shapes follow the reference's tensors:

* ``(b f)`` activations: ``(B*f, N, C)`` rows ordered batch-major, frame-minor (attention.py:94)
* ``(b d)`` activations: ``(B*N, f, C)`` (the temporal rearrange, attention.py:263)
"""
from __future__ import annotations

import ctypes
import json
import os
from typing import Optional

import torch
import torch.nn.functional as F

from . import _lib
from ._lib import check

_DT = {torch.float32: _lib.F32, torch.bfloat16: _lib.BF16}


def _dtype(*ts):
    d = ts[0].dtype
    for t in ts:
        if t.dtype != d:
            raise TypeError(f"dtype mismatch: {[x.dtype for x in ts]}")
        if not t.is_cuda:
            raise RuntimeError("vp2p ops run on the GPU only (tensor on %s)" % t.device)
        if t.stride(-1) != 1:
            raise ValueError("channel dimension must be contiguous")
    if d not in _DT:
        raise TypeError(f"unsupported dtype {d}")
    return _DT[d]


def version_key(*ts):
    """Key of the current contents of ``ts`` for a derived-tensor cache: each tensor's storage and
    version counter (None for an absent tensor).  None when one of them is an inference tensor
    (``torch.inference_mode``): those have no version counter, so an in-place write could not be
    detected -- the caller then recomputes and caches nothing."""
    out = []
    for t in ts:
        if t is None:
            out.append(None)
        elif t.is_inference():
            return None
        else:
            out.append((t.data_ptr(), t._version, t.dtype, t.device))
    return tuple(out)


def _stream():
    """The current HIP stream of the current device (the raw handle: no Stream object per launch)."""
    return ctypes.c_void_p(torch._C._cuda_getCurrentRawStream(torch._C._cuda_getDevice()))


def _ptr(t: Optional[torch.Tensor]):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _bf_strides(t: torch.Tensor, frames: int):
    """(b, f, n) element strides of a '(b f) n c' tensor."""
    s0, s1 = t.stride(0), t.stride(1)
    return frames * s0, s0, s1


def _bd_strides(t: torch.Tensor, tokens: int):
    """(b, f, n) element strides of a '(b d) f c' tensor."""
    s0, s1 = t.stride(0), t.stride(1)
    return tokens * s0, s1, s0


# ----------------------------------------------------------------------------------------------
def frame_attention(q: torch.Tensor, k0: torch.Tensor, v0: torch.Tensor, frames: int, heads: int,
                    scale: Optional[float] = None, out: Optional[torch.Tensor] = None,
                    lse: Optional[torch.Tensor] = None, q_prescaled: bool = False) -> torch.Tensor:
    """FrameAttention core (attention.py:282-322).  q: (B*f, N, C); k0, v0: frame-0 keys/values
    (B, Nk, C) -- or full (B*f, Nk, C) tensors, of which only frame 0 is read.  ``lse``: optional
    (B, heads, f*N) fp32 output of each row's log2-sum-exp2 (saved for the backward).
    ``q_prescaled``: q already holds q * scale * log2(e) (see ``frame_query_scale``); K1 then runs
    its folded-max form at head_dim 40."""
    dt = _dtype(q, k0, v0)
    Bf, N, C = q.shape
    B = Bf // frames
    if B * frames != Bf or C % heads:
        raise ValueError("bad shapes")
    if out is None:
        out = torch.empty_like(q, memory_format=torch.contiguous_format)
    d = C // heads
    k_sb = k0.stride(0) * (frames if k0.shape[0] == Bf else 1)
    v_sb = v0.stride(0) * (frames if v0.shape[0] == Bf else 1)
    if k0.shape[0] not in (B, Bf) or v0.shape[0] != k0.shape[0]:
        raise ValueError("k0/v0 must be (B, Nk, C) or (B*f, Nk, C)")
    q_sb, q_sf, q_sn = _bf_strides(q, frames)
    o_sb, o_sf, o_sn = _bf_strides(out, frames)
    a = _lib.FrameAttnArgs(_ptr(q), _ptr(k0), _ptr(v0), _ptr(out), q_sb, q_sf, q_sn,
                           k_sb, k0.stride(1), v_sb, v0.stride(1), o_sb, o_sf, o_sn,
                           B, frames, N, k0.shape[1], heads, d,
                           float(d ** -0.5 if scale is None else scale), dt, _ptr(lse), int(bool(q_prescaled)))
    if lse is not None and (lse.dtype != torch.float32 or not lse.is_contiguous()
                            or lse.numel() != B * heads * frames * N):
        raise ValueError("lse must be a contiguous fp32 (B, heads, f*N) tensor")
    check(_lib.load().vp2p_frame_attn_fwd(ctypes.byref(a), _stream()), "vp2p_frame_attn_fwd")
    return out


def frame_query_scale(head_dim: int, scale: Optional[float] = None) -> float:
    """The factor a caller folds into q for ``frame_attention(..., q_prescaled=True)``:
    softmax scale (head_dim ** -0.5 by default) times log2(e)."""
    return float(head_dim ** -0.5 if scale is None else scale) * 1.4426950408889634


def frame_attention_bwd(q, k, v, o, dout, lse, frames: int, heads: int, scale: float,
                        dq: torch.Tensor, dk: torch.Tensor, dv: torch.Tensor) -> None:
    """Backward of ``frame_attention`` (K1b): fills dq (like q) and dk, dv (like k, v).  q, o, dout
    and dq must share their (b f, n) strides; k, v, dk and dv theirs (e.g. views of one K|V
    buffer and of its gradient)."""
    dt = _dtype(q, k, v, o, dout, dq, dk, dv)
    Bf, N, C = q.shape
    B = Bf // frames
    for t in (o, dout, dq):
        if t.shape != q.shape or t.stride() != q.stride():
            raise ValueError("q, o, dout, dq must share shape and strides")
    for t in (v, dk, dv):
        if t.shape != k.shape or t.stride() != k.stride():
            raise ValueError("k, v, dk, dv must share shape and strides")
    if k.shape[0] != B:
        raise ValueError("k/v must be (B, Nk, C)")
    q_sb, q_sf, q_sn = _bf_strides(q, frames)
    a = _lib.FrameAttnBwdArgs(_ptr(q), _ptr(k), _ptr(v), _ptr(o), _ptr(dout), _ptr(lse), _ptr(dq), _ptr(dk),
                              _ptr(dv), None, q_sb, q_sf, q_sn, k.stride(0), k.stride(1),
                              B, frames, N, k.shape[1], heads, C // heads, float(scale), dt)
    lib = _lib.load()
    nbytes = lib.vp2p_frame_attn_bwd_workspace_bytes(ctypes.byref(a))
    if nbytes < 0:
        check(int(nbytes), "vp2p_frame_attn_bwd_workspace_bytes")
    ws = torch.empty(max(int(nbytes), 16), dtype=torch.uint8, device=q.device)
    a.workspace = ws.data_ptr()
    check(lib.vp2p_frame_attn_bwd(ctypes.byref(a), _stream()), "vp2p_frame_attn_bwd")


def temporal_attention_bwd(q, k, v, dout, frames: int, heads: int, scale: float, dq, dk, dv) -> None:
    """Backward of the plain hooked temporal attention (K3b) on '(b f) n c' tensors (B*f, N, C)."""
    dt = _dtype(q, k, v, dout, dq, dk, dv)
    Bf, N, C = q.shape
    st = []
    for t in (q, k, v, dout, dq, dk, dv):
        if t.shape != q.shape:
            raise ValueError("temporal backward: shape mismatch")
        st += list(_bf_strides(t, frames))
    a = _lib.TemporalAttnBwdArgs(_ptr(q), _ptr(k), _ptr(v), _ptr(dout), _ptr(dq), _ptr(dk), _ptr(dv), *st,
                                 Bf // frames, frames, N, heads, C // heads, float(scale), dt)
    check(_lib.load().vp2p_temporal_attn_bwd(ctypes.byref(a), _stream()), "vp2p_temporal_attn_bwd")


# ----------------------------------------------------------------------------------------------
class CrossEditPlan:
    """Device-resident descriptor of an AttentionControlEdit for the fused cross kernel.

    Built once per controller (host work happens here, not per call): the per-step word alphas
    (cross_replace_alpha, run_videop2p.py:325), the mapper as CSC (Replace) or a gather index
    (Refine), the equalizer (Reweight) and LocalBlend's word weights."""

    def __init__(self, prompts: int, edit_mode: int, reweight: bool, alpha_steps: torch.Tensor,
                 mapper=None, refine_alpha=None, equalizer=None, lb_word_alpha=None,
                 device="cuda", tokens_kv: int = 77):
        self.prompts = prompts
        self.edit_mode = edit_mode
        self.reweight = bool(reweight)
        self.tokens_kv = tokens_kv
        dev = torch.device(device)
        # (steps+1, P-1, 77) float32
        self.alpha_steps = alpha_steps.reshape(alpha_steps.shape[0], prompts - 1, -1).float().contiguous().to(dev)
        self.map_ptr = self.map_idx = self.map_val = self.refine_alpha = None
        if edit_mode == _lib.EDIT_REPLACE:
            m = torch.as_tensor(mapper, dtype=torch.float32).reshape(prompts - 1, tokens_kv, tokens_kv)
            ptr, idx, val = [], [], []
            for pe in range(prompts - 1):
                base = len(idx)
                ptr.append(base)
                col_ptr = [base]
                for w in range(tokens_kv):
                    nz = torch.nonzero(m[pe, :, w]).flatten().tolist()
                    idx.extend(nz)
                    val.extend(m[pe, nz, w].tolist())
                    col_ptr.append(len(idx))
                ptr[-1:] = col_ptr
            self.map_ptr = torch.tensor(ptr, dtype=torch.int32, device=dev)
            self.map_idx = torch.tensor(idx or [0], dtype=torch.int32, device=dev)
            self.map_val = torch.tensor(val or [0.0], dtype=torch.float32, device=dev)
        elif edit_mode == _lib.EDIT_REFINE:
            mp = torch.as_tensor(mapper, dtype=torch.int64).reshape(prompts - 1, tokens_kv)
            self.map_idx = (mp % tokens_kv).to(torch.int32).contiguous().to(dev)  # -1 -> last word
            self.refine_alpha = torch.as_tensor(refine_alpha, dtype=torch.float32).reshape(
                prompts - 1, tokens_kv).contiguous().to(dev)
        self.equalizer = (None if equalizer is None else
                          torch.as_tensor(equalizer, dtype=torch.float32).reshape(-1)[:tokens_kv].contiguous().to(dev))
        # (sets, prompts, 77): set 0 = LocalBlend's blend words, set 1 = its substruct_words (optional)
        self.lb_word_alpha = (None if lb_word_alpha is None else
                              torch.as_tensor(lb_word_alpha, dtype=torch.float32).reshape(-1, prompts, tokens_kv)
                              .contiguous().to(dev))
        self.lb_sets = 0 if self.lb_word_alpha is None else self.lb_word_alpha.shape[0]
        if self.lb_sets > 2:
            raise ValueError("LocalBlend word weights: at most 2 sets (blend words, substruct words)")

    def alpha_ptr(self, step: int):
        return ctypes.c_void_p(self.alpha_steps[step].data_ptr())


def cross_kv_prep(k: torch.Tensor, v: torch.Tensor, heads: int) -> torch.Tensor:
    dt = _dtype(k, v)
    B, nkv, C = k.shape
    lib = _lib.load()
    nbytes = lib.vp2p_cross_kv_workspace_bytes(B, nkv, heads, C // heads, dt)
    if nbytes < 0:
        check(int(nbytes), "vp2p_cross_kv_workspace_bytes")
    ws = torch.empty(int(nbytes), dtype=torch.uint8, device=k.device)
    check(lib.vp2p_cross_kv_prep(_ptr(k), _ptr(v), k.stride(0), k.stride(1), v.stride(0), v.stride(1),
                                 B, nkv, heads, C // heads, dt, _ptr(ws), _stream()), "vp2p_cross_kv_prep")
    return ws


def cross_attention_p2p(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, frames: int, heads: int,
                        plan: Optional[CrossEditPlan] = None, step: int = 0, edit: bool = True,
                        lb_acc: Optional[torch.Tensor] = None, probs_out: Optional[torch.Tensor] = None,
                        scale: Optional[float] = None, out: Optional[torch.Tensor] = None,
                        prompts: int = 0, cond_only: bool = False,
                        kv_ws: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Hooked attn2 (ptp_utils.py:196-221) with the controller edit fused.  q: (B*f, N, C);
    k, v: the projected context (B, Nk, C) shared by all frames of a batch row.  ``cond_only``: the
    batch is only the conditional half (B = prompts; a CFG-split rank).  ``kv_ws``: k / v already laid
    out by ``cross_kv_prep`` (the caller caches it while the context is unchanged)."""
    dt = _dtype(q, k, v)
    Bf, N, C = q.shape
    B = Bf // frames
    if k.shape[0] != B:
        raise ValueError("k/v must be (B, Nk, C)")
    d = C // heads
    nkv = k.shape[1]
    ws = cross_kv_prep(k, v, heads) if kv_ws is None else kv_ws
    if out is None:
        out = torch.empty_like(q, memory_format=torch.contiguous_format)
    q_sb, q_sf, q_sn = _bf_strides(q, frames)
    o_sb, o_sf, o_sn = _bf_strides(out, frames)
    P = plan.prompts if plan is not None else prompts
    sets = 1
    if lb_acc is not None:      # (P, f, N), or (sets, P, f, N) with the substruct_words set
        sets = plan.lb_sets if plan is not None else 0
        shape = (P, frames, N) if sets == 1 else (sets, P, frames, N)
        if sets < 1 or tuple(lb_acc.shape) != shape or not lb_acc.is_contiguous() or lb_acc.dtype != torch.float32:
            raise ValueError(f"lb_acc must be a contiguous fp32 {shape} tensor")
    mode = plan.edit_mode if (plan is not None and edit) else _lib.EDIT_NONE
    rew = int(plan.reweight) if (plan is not None and edit) else 0
    a = _lib.CrossAttnArgs(_ptr(q), _ptr(ws), _ptr(out), q_sb, q_sf, q_sn, o_sb, o_sf, o_sn,
                           B, frames, N, nkv, heads, d, float(d ** -0.5 if scale is None else scale), dt,
                           P, mode, rew,
                           plan.alpha_ptr(step) if plan is not None else None,
                           _ptr(plan.map_ptr) if plan is not None else None,
                           _ptr(plan.map_idx) if plan is not None else None,
                           _ptr(plan.map_val) if plan is not None else None,
                           _ptr(plan.refine_alpha) if plan is not None else None,
                           _ptr(plan.equalizer) if plan is not None else None,
                           _ptr(lb_acc), _ptr(plan.lb_word_alpha) if (plan is not None and lb_acc is not None) else None,
                           _ptr(probs_out), None, sets, int(cond_only))
    lb_ws = None
    if lb_acc is not None:       # per-head partials, reduced in head order by the library's second pass
        lb_ws = torch.empty(sets * P * heads * frames * N, device=q.device, dtype=torch.float32)
        a.lb_ws = _ptr(lb_ws)
    check(_lib.load().vp2p_cross_attn_p2p_fwd(ctypes.byref(a), _stream()), "vp2p_cross_attn_p2p_fwd")
    return out


def temporal_attention_p2p(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, frames: int, heads: int,
                           prompts: int = 0, self_replace: bool = False,
                           probs_out: Optional[torch.Tensor] = None, scale: Optional[float] = None,
                           out: Optional[torch.Tensor] = None, cond_only: bool = False) -> torch.Tensor:
    """Hooked attn_temp with replace_self_attention on '(b f) n c' tensors (B*f, N, C): the
    temporal rearrange of attention.py:263 is expressed through strides, never materialised."""
    dt = _dtype(q, k, v)
    Bf, N, C = q.shape
    B = Bf // frames
    st = lambda t: _bf_strides(t, frames)  # noqa: E731
    if out is None:
        out = torch.empty_like(q, memory_format=torch.contiguous_format)
    d = C // heads
    a = _lib.TemporalAttnArgs(_ptr(q), _ptr(k), _ptr(v), _ptr(out), *st(q), *st(k), *st(v), *st(out),
                              B, frames, N, heads, d, float(d ** -0.5 if scale is None else scale), dt,
                              prompts, int(self_replace), _ptr(probs_out), int(cond_only))
    check(_lib.load().vp2p_temporal_attn_p2p_fwd(ctypes.byref(a), _stream()), "vp2p_temporal_attn_p2p_fwd")
    return out


def temporal_attention_p2p_bd(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, batch: int, heads: int,
                              prompts: int = 0, self_replace: bool = False,
                              probs_out: Optional[torch.Tensor] = None, scale: Optional[float] = None,
                              out: Optional[torch.Tensor] = None, cond_only: bool = False) -> torch.Tensor:
    """Same op on the reference's '(b d) f c' tensors (B*N, f, C)."""
    dt = _dtype(q, k, v)
    BN, F, C = q.shape
    N = BN // batch
    if out is None:
        out = torch.empty_like(q, memory_format=torch.contiguous_format)
    st = lambda t: _bd_strides(t, N)  # noqa: E731
    d = C // heads
    a = _lib.TemporalAttnArgs(_ptr(q), _ptr(k), _ptr(v), _ptr(out), *st(q), *st(k), *st(v), *st(out),
                              batch, F, N, heads, d, float(d ** -0.5 if scale is None else scale), dt,
                              prompts, int(self_replace), _ptr(probs_out), int(cond_only))
    check(_lib.load().vp2p_temporal_attn_p2p_fwd(ctypes.byref(a), _stream()), "vp2p_temporal_attn_p2p_fwd")
    return out


# ----------------------------------------------------------------------------------------------
def step_fused(noise: torch.Tensor, latents: torch.Tensor, consts, guidance: float = 7.5, cfg: bool = True,
               fast: bool = False, lb_acc: Optional[torch.Tensor] = None, lb_hw=(16, 16),
               lb_count: float = 40.0, lb_th: float = 0.3, out: Optional[torch.Tensor] = None,
               lb_sub_th: float = 0.3, mask_out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """CFG + DDIM update + LocalBlend in one launch.  noise: (2P or P, C, f, H, W) bf16/f32,
    latents: (P, C, f, H, W) fp32, consts = (c1, c2, c3, c4) float32 scalars.  ``lb_acc``: the
    LocalBlend sums, (P, f, h*w) or (sets, P, f, h*w) with set 1 = the substruct_words sum
    (thresholded at ``lb_sub_th`` without pooling, run_videop2p.py:149-151).  ``mask_out``: optional
    contiguous uint8 (P, f, H, W) that receives the blend mask the launch applied (when lb_acc is set)."""
    if not (noise.is_cuda and latents.is_cuda):
        raise RuntimeError("step_fused runs on the GPU only")
    if latents.dtype != torch.float32 or not latents.is_contiguous() or not noise.is_contiguous():
        raise ValueError("latents must be contiguous fp32, noise contiguous")
    P, C, F, H, W = latents.shape
    if noise.shape[0] != (2 * P if cfg else P) or tuple(noise.shape[1:]) != (C, F, H, W):
        raise ValueError(f"noise shape {tuple(noise.shape)} vs latents {tuple(latents.shape)}")
    if out is None:
        out = torch.empty_like(latents)
    c1, c2, c3, c4 = (float(c) for c in consts)
    lb_sub = None
    if lb_acc is not None:
        if lb_acc.dim() == 4:
            if lb_acc.shape[0] == 2:
                lb_sub = lb_acc[1]
            lb_acc = lb_acc[0]
        if tuple(lb_acc.shape) != (P, F, int(lb_hw[0]) * int(lb_hw[1])) or not lb_acc.is_contiguous():
            raise ValueError(f"lb_acc: expected contiguous {(P, F, int(lb_hw[0]) * int(lb_hw[1]))}, "
                             f"got {tuple(lb_acc.shape)}")
    a = _lib.StepArgs(_ptr(noise), _DT[noise.dtype], _ptr(latents), _ptr(out), P, C, F, H, W,
                      int(cfg), int(fast), float(guidance), c1, c2, c3, c4,
                      _ptr(lb_acc), int(lb_hw[0]), int(lb_hw[1]), float(lb_count), float(lb_th),
                      _ptr(lb_sub), float(lb_sub_th))
    if mask_out is not None:
        if (mask_out.dtype != torch.uint8 or not mask_out.is_contiguous() or not mask_out.is_cuda
                or tuple(mask_out.shape) != (P, F, H, W)):
            raise ValueError(f"mask_out must be a contiguous uint8 device tensor of shape {(P, F, H, W)}")
        a.mask_out = _ptr(mask_out)
    check(_lib.load().vp2p_step_fused(ctypes.byref(a), _stream()), "vp2p_step_fused")
    return out


def nulltext_loss(noise_uncond: torch.Tensor, noise_cond: torch.Tensor, latents: torch.Tensor,
                  latents_prev: torch.Tensor, consts, guidance: float = 7.5):
    """Null-text inner loss mean((prev_step(u + g (c - u)) - x_prev)^2) and its gradient w.r.t. u
    (run_videop2p.py:594-599) in one pass.  Returns (loss (0-d fp32 tensor), grad like u)."""
    for t in (noise_uncond, noise_cond, latents, latents_prev):
        if not t.is_cuda or not t.is_contiguous():
            raise ValueError("nulltext_loss: contiguous device tensors expected")
    n = noise_uncond.numel()
    if noise_cond.dtype != noise_uncond.dtype or any(t.numel() != n for t in (noise_cond, latents, latents_prev)):
        raise ValueError("nulltext_loss: shape/dtype mismatch")
    if latents.dtype != torch.float32 or latents_prev.dtype != torch.float32:
        raise ValueError("nulltext_loss: latents must be fp32")
    lib = _lib.load()
    grad = torch.empty_like(noise_uncond)
    parts = torch.empty(lib.vp2p_nulltext_loss_partials() + 1, device=latents.device, dtype=torch.float32)
    c1, c2, c3, c4 = (float(c) for c in consts)
    a = _lib.NullTextLossArgs(_ptr(noise_uncond), _ptr(noise_cond), _DT[noise_uncond.dtype], _ptr(latents),
                              _ptr(latents_prev), _ptr(grad), _ptr(parts[1:]), _ptr(parts), n, float(guidance),
                              c1, c2, c3, c4)
    check(lib.vp2p_nulltext_loss(ctypes.byref(a), _stream()), "vp2p_nulltext_loss")
    return parts[0], grad


# ----------------------------------------------------------------------------------------------
# Non-attention UNet path (K7-K9)
# ----------------------------------------------------------------------------------------------
def _rows_view(x: torch.Tensor) -> torch.Tensor:
    """A channels-last activation ((Bf, C, H, W) in channels_last memory, or contiguous (..., C)) as
    the (rows, C) matrix the kernels read; raises if the memory is not laid out that way."""
    if x.dim() == 4:
        if not x.is_contiguous(memory_format=torch.channels_last):
            raise ValueError("expected a channels_last (Bf, C, H, W) tensor")
        return x.permute(0, 2, 3, 1).reshape(-1, x.shape[1])
    if not x.is_contiguous():
        raise ValueError("expected a contiguous (..., C) tensor")
    return x.reshape(-1, x.shape[-1])


def _gn_args(x, num_groups, weight, bias, eps, frames, silu, add, out, x2=None):
    Bf, C = x.shape[0], x.shape[1] + (0 if x2 is None else x2.shape[1])
    xm = _rows_view(x)
    x2m = None
    if x2 is not None:
        x2m = _rows_view(x2)
        if x2.dtype != x.dtype or x2.shape[0] != Bf or x2.shape[2:] != x.shape[2:]:
            raise ValueError("x2 must match x in dtype, samples and spatial size")
    dt = _dtype(xm)
    if Bf % frames:
        raise ValueError(f"{Bf} samples are not a multiple of {frames} frames")
    rows = xm.shape[0] // Bf
    ym = _rows_view(out) if out is not None else None
    for t in (weight, bias, add):
        if t is not None and (t.dtype != x.dtype or not t.is_contiguous() or not t.is_cuda):
            raise ValueError("weight/bias/add must be contiguous device tensors of the activation dtype")
    if add is not None and tuple(add.shape) != (Bf, C):
        raise ValueError(f"add must be (Bf, C) = {(Bf, C)}, got {tuple(add.shape)}")
    a = _lib.GroupNormArgs(_ptr(xm), _ptr(add), _ptr(ym), _ptr(weight), _ptr(bias), None, Bf // frames, frames,
                           rows, C, num_groups, float(eps), int(silu), dt)
    if x2 is not None:
        a.x2, a.channels2 = _ptr(x2m), x2.shape[1]
    return a


# Partial sets from which the finalize launch (~5 us) pays for itself: below it every apply block
# merges the few partials itself (profiles/r02_gn_finalize_ab.jsonl: 8x8 latents, 22 partials:
# 8.6 us merged in the apply vs 5.3 + 5.8; 64x64 at 320 channels, 249 partials: 44.0 vs 6.3 + 31.9).
GN_FINALIZE_MIN_PARTS = 128


_GN_PARTS = {}      # (samples, frames, rows, channels, groups) -> partial sets of the stats launch


def _gn_parts(lib, a) -> int:
    key = (a.batch, a.frames, a.rows, a.channels, a.groups)
    parts = _GN_PARTS.get(key)
    if parts is None:
        parts = lib.vp2p_group_norm_parts(ctypes.byref(a))
        if parts < 0:
            check(parts, "vp2p_group_norm_parts")
        _GN_PARTS[key] = parts
    return parts


def group_norm(x: torch.Tensor, num_groups: int, weight: Optional[torch.Tensor], bias: Optional[torch.Tensor],
               eps: float, frames: int, silu: bool = False, add: Optional[torch.Tensor] = None,
               shard=None, out: Optional[torch.Tensor] = None, return_stats: bool = False,
               x2: Optional[torch.Tensor] = None):
    """GroupNorm of a ``(b f) c h w`` channels-last tensor with statistics over (c/G, f, h, w) of
    each batch element (tuneavideo resnet.py:142,158; frames=1: per-frame, attention.py:110),
    optionally on x + add[(b f), c] (the resnet's h + temb, resnet.py:149-156) and followed by SiLU.
    ``shard``: a FrameShard whose ranks hold the other frames; their partial statistics are
    gathered between the two kernels.  ``return_stats``: also return (partials, nsets), the
    statistics the backward needs.  ``x2``: normalise torch.cat([x, x2], dim=1) (channels-last,
    forward only) without writing the cat."""
    Bf = x.shape[0]
    if out is None:
        if x2 is None:
            out = torch.empty_like(x)
        else:
            out = torch.empty((Bf, x.shape[1] + x2.shape[1]) + tuple(x.shape[2:]), device=x.device, dtype=x.dtype,
                              memory_format=torch.channels_last)
    a = _gn_args(x, num_groups, weight, bias, eps, frames, silu, add, out, x2)
    lib = _lib.load()
    parts = _gn_parts(lib, a)
    partials = torch.empty((Bf // frames) * parts * num_groups * 3, device=x.device, dtype=torch.float32)
    a.partials = partials.data_ptr()
    s = _stream()
    check(lib.vp2p_group_norm_stats(ctypes.byref(a), s), "vp2p_group_norm_stats")
    nsets = 1
    if shard is not None and shard.world > 1 and not return_stats:
        # frames sharded: each rank merges its own partials into one (count, mean, M2) per
        # (batch, group) and the ranks exchange those (B*G*12 bytes, not B*parts*G*12)
        tri = torch.empty((Bf // frames) * num_groups * 3, device=x.device, dtype=torch.float32)
        check(lib.vp2p_group_norm_merge(ctypes.byref(a), _ptr(partials), _ptr(tri), s), "vp2p_group_norm_merge")
        tri = shard.all_gather_flat(tri)
        st = torch.empty((Bf // frames) * num_groups * 2, device=x.device, dtype=torch.float32)
        check(lib.vp2p_group_norm_finalize_merged(ctypes.byref(a), _ptr(tri), shard.world, _ptr(st), s),
              "vp2p_group_norm_finalize_merged")
        check(lib.vp2p_group_norm_apply_stats(ctypes.byref(a), _ptr(st), s), "vp2p_group_norm_apply_stats")
        return out
    if shard is not None and shard.world > 1:
        partials = shard.all_gather_flat(partials)     # the backward re-reads every rank's partials
        nsets = shard.world
    if parts * nsets >= GN_FINALIZE_MIN_PARTS:
        # one finalize launch merges the partials into (mean, rstd) per (batch, group); the apply
        # blocks then read 2 floats per group instead of each merging every partial
        st = torch.empty((Bf // frames) * num_groups * 2, device=x.device, dtype=torch.float32)
        check(lib.vp2p_group_norm_finalize(ctypes.byref(a), _ptr(partials), nsets, _ptr(st), s),
              "vp2p_group_norm_finalize")
        check(lib.vp2p_group_norm_apply_stats(ctypes.byref(a), _ptr(st), s), "vp2p_group_norm_apply_stats")
    else:
        check(lib.vp2p_group_norm_apply(ctypes.byref(a), _ptr(partials), nsets, s), "vp2p_group_norm_apply")
    if return_stats:
        return out, (partials, nsets)
    return out


def group_norm_bwd(x: torch.Tensor, dy: torch.Tensor, stats, num_groups: int, weight, bias, eps: float,
                   frames: int, silu: bool = False, add: Optional[torch.Tensor] = None, shard=None) -> torch.Tensor:
    """Input gradient of ``group_norm`` (K7b) given the forward's ``stats`` = (partials, nsets);
    dy and the result are channels-last like x.  ``shard``: the FrameShard of the forward -- the
    per-chunk backward partials of every rank are gathered before the apply kernel."""
    partials, nsets = stats
    if not dy.is_contiguous(memory_format=torch.channels_last):
        dy = dy.contiguous(memory_format=torch.channels_last)
    dx = torch.empty_like(x, memory_format=torch.channels_last)
    a = _gn_args(x, num_groups, weight, bias, eps, frames, silu, add, dx)   # y is not read by the backward
    lib = _lib.load()
    parts = lib.vp2p_group_norm_parts(ctypes.byref(a))
    if parts < 0:
        check(parts, "vp2p_group_norm_parts")
    bpart = torch.empty((x.shape[0] // frames) * parts * num_groups * 2, device=x.device, dtype=torch.float32)
    s = _stream()
    dym = _rows_view(dy)
    check(lib.vp2p_group_norm_bwd_reduce(ctypes.byref(a), _ptr(partials), nsets, _ptr(dym), _ptr(bpart), s),
          "vp2p_group_norm_bwd_reduce")
    bsets = 1
    if shard is not None and shard.world > 1:
        bpart = shard.all_gather_flat(bpart)
        bsets = shard.world
    check(lib.vp2p_group_norm_bwd_apply(ctypes.byref(a), _ptr(partials), nsets, _ptr(dym), _ptr(bpart), bsets,
                                        _ptr(_rows_view(dx)), s), "vp2p_group_norm_bwd_apply")
    return dx


def layer_norm(x: torch.Tensor, weight: Optional[torch.Tensor], bias: Optional[torch.Tensor], eps: float,
               out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """nn.LayerNorm over the last (channel) axis (attention.py:200-216)."""
    if not x.is_contiguous():
        x = x.contiguous()
    dt = _dtype(x)
    C = x.shape[-1]
    out = torch.empty_like(x) if out is None else out
    for t in (weight, bias):
        if t is not None and (t.dtype != x.dtype or not t.is_contiguous()):
            raise ValueError("weight/bias must be contiguous tensors of the activation dtype")
    a = _lib.LayerNormArgs(_ptr(x), _ptr(out), _ptr(weight), _ptr(bias), x.numel() // C, C, float(eps), dt)
    check(_lib.load().vp2p_layer_norm_fwd(ctypes.byref(a), _stream()), "vp2p_layer_norm_fwd")
    return out


def add_layer_norm(h: torch.Tensor, x: torch.Tensor, weight: Optional[torch.Tensor], bias: Optional[torch.Tensor],
                   eps: float):
    """The transformer block's residual add fused into the next LayerNorm (K8 + add):
    returns (s, y) with s = h + x (rounded to the dtype, written over ``h``) and y = LayerNorm(s)."""
    if not h.is_contiguous() or not x.is_contiguous() or h.shape != x.shape:
        raise ValueError("add_layer_norm: h and x must be contiguous tensors of one shape")
    dt = _dtype(h, x)
    C = h.shape[-1]
    for t in (weight, bias):
        if t is not None and (t.dtype != h.dtype or not t.is_contiguous()):
            raise ValueError("weight/bias must be contiguous tensors of the activation dtype")
    y = torch.empty_like(h)
    a = _lib.LayerNormArgs(_ptr(h), _ptr(y), _ptr(weight), _ptr(bias), h.numel() // C, C, float(eps), dt)
    check(_lib.load().vp2p_add_layer_norm_fwd(ctypes.byref(a), _ptr(x), _ptr(h), _stream()),
          "vp2p_add_layer_norm_fwd")
    return h, y


def geglu(h: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """GEGLU gate a * gelu(g) of a (..., 2*inner) projection (diffusers 0.11.1 GEGLU.forward)."""
    if not h.is_contiguous():
        h = h.contiguous()
    dt = _dtype(h)
    inner = h.shape[-1] // 2
    if out is None:
        out = torch.empty(*h.shape[:-1], inner, device=h.device, dtype=h.dtype)
    check(_lib.load().vp2p_geglu_fwd(_ptr(h), _ptr(out), h.numel() // (2 * inner), inner, dt, _stream()),
          "vp2p_geglu_fwd")
    return out


def layer_norm_bwd(x: torch.Tensor, dy: torch.Tensor, weight: Optional[torch.Tensor], eps: float) -> torch.Tensor:
    """Input gradient of ``layer_norm`` (K8b)."""
    x = x.contiguous()
    dy = dy.contiguous()
    dt = _dtype(x, dy)
    C = x.shape[-1]
    dx = torch.empty_like(x)
    a = _lib.LayerNormArgs(_ptr(x), None, _ptr(weight), None, x.numel() // C, C, float(eps), dt)
    check(_lib.load().vp2p_layer_norm_bwd(ctypes.byref(a), _ptr(dy), _ptr(dx), _stream()), "vp2p_layer_norm_bwd")
    return dx


def geglu_bwd(h: torch.Tensor, dy: torch.Tensor) -> torch.Tensor:
    """Gradient of ``geglu`` w.r.t. its (..., 2*inner) input (K9b)."""
    h = h.contiguous()
    dy = dy.contiguous()
    dt = _dtype(h, dy)
    inner = h.shape[-1] // 2
    dh = torch.empty_like(h)
    check(_lib.load().vp2p_geglu_bwd(_ptr(h), _ptr(dy), _ptr(dh), h.numel() // (2 * inner), inner, dt, _stream()),
          "vp2p_geglu_bwd")
    return dh


def _conv_args(x: torch.Tensor, weight: torch.Tensor, bias, residual, y, stride: int, padding: int,
               upsample: bool = False, x2: Optional[torch.Tensor] = None):
    N, Cin, H, W = x.shape
    if x2 is not None:
        Cin += x2.shape[1]
    if upsample:
        H, W = 2 * H, 2 * W
    Cout, _, KH, KW = weight.shape
    Ho = (H + 2 * padding - KH) // stride + 1
    Wo = (W + 2 * padding - KW) // stride + 1
    dt = _lib.BF16 if x.dtype == torch.bfloat16 else -1
    a = _lib.ConvArgs(_ptr(x), _ptr(weight), _ptr(bias), _ptr(residual), _ptr(y), N, H, W, Cin, Cout, Ho, Wo,
                      KH if KH == KW else -1, stride, padding, dt)
    a.upsample = 1 if upsample else 0
    if x2 is not None:
        a.x2, a.cin2 = _ptr(x2), x2.shape[1]
    return a, (N, Cout, Ho, Wo)


def conv2d_supported(x: torch.Tensor, weight: torch.Tensor, stride: int = 1, padding: int = 0,
                     upsample: bool = False, x2: Optional[torch.Tensor] = None) -> bool:
    """True when K10 covers this convolution: bf16, channels-last, 1x1 / 3x3 'same' padding, stride
    1 or 2, Cin % 64 == 0, Cout % 160 == 0 (every resnet / up/down-sample conv of the SD-1.5 UNet
    except conv_in / conv_out)."""
    if x.dtype != torch.bfloat16 or weight.dtype != torch.bfloat16 or not x.is_cuda or x.dim() != 4:
        return False
    if not x.is_contiguous(memory_format=torch.channels_last):
        return False
    if x2 is not None and (x2.dtype != x.dtype or x2.shape[0] != x.shape[0] or x2.shape[2:] != x.shape[2:]
                           or not x2.is_contiguous(memory_format=torch.channels_last)):
        return False
    a, _ = _conv_args(x, weight, None, None, None, stride, padding, upsample, x2)
    return bool(_lib.load().vp2p_conv2d_supported(ctypes.byref(a)))


_CONV_WS = {}       # conv geometry -> split-K workspace bytes (a pure function of the shape)


def conv2d(x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor] = None, stride: int = 1,
           padding: int = 0, residual: Optional[torch.Tensor] = None, upsample: bool = False,
           x2: Optional[torch.Tensor] = None, img_add: Optional[torch.Tensor] = None) -> torch.Tensor:
    """K10: nn.Conv2d on channels-last bf16 with the bias and an optional residual add fused
    (``residual + conv(x)``, the resnet shortcut add of resnet.py:196-205) or a per-image vector
    added after the bias (``img_add`` (N, Cout): the resnet's h + temb, resnet.py:149-156).  Returns a
    channels-last (N, Cout, Ho, Wo) tensor.  Raises for shapes K10 does not cover (see
    ``conv2d_supported``)."""
    if not x.is_contiguous(memory_format=torch.channels_last):
        raise ValueError("conv2d: x must be channels-last contiguous")
    w = weight if weight.is_contiguous(memory_format=torch.channels_last) else \
        weight.contiguous(memory_format=torch.channels_last)
    if bias is not None and (bias.dtype != x.dtype or not bias.is_contiguous()):
        bias = bias.to(x.dtype).contiguous()
    if x2 is not None and not x2.is_contiguous(memory_format=torch.channels_last):
        raise ValueError("conv2d: x2 must be channels-last contiguous")
    a, shape = _conv_args(x, w, bias, None, None, stride, padding, upsample, x2)
    y = torch.empty(shape, device=x.device, dtype=x.dtype, memory_format=torch.channels_last)
    if residual is not None:
        if residual.shape != y.shape or residual.dtype != y.dtype:
            raise ValueError("conv2d: residual must match the output")
        if not residual.is_contiguous(memory_format=torch.channels_last):
            residual = residual.contiguous(memory_format=torch.channels_last)
        a.residual = _ptr(residual)
    if img_add is not None:
        if tuple(img_add.shape) != (shape[0], shape[1]) or img_add.dtype != y.dtype:
            raise ValueError("conv2d: img_add must be (N, Cout) of the output dtype")
        img_add = img_add.contiguous()
        a.img_add = _ptr(img_add)
    a.y = _ptr(y)
    lib = _lib.load()
    wkey = (a.batch, a.in_h, a.in_w, a.cin, a.cout, a.kernel, a.stride, a.pad, a.upsample, a.cin2, a.epilogue)
    wsb = _CONV_WS.get(wkey)
    if wsb is None:
        wsb = _CONV_WS[wkey] = lib.vp2p_conv2d_workspace_bytes(ctypes.byref(a))
    ws = None
    if wsb > 0:      # split-K slices (small-M shapes); from the caching allocator, no sync
        ws = torch.empty(wsb // 4, device=x.device, dtype=torch.float32)
        a.workspace = _ptr(ws)
    check(lib.vp2p_conv2d_fwd(ctypes.byref(a), _stream()), "vp2p_conv2d_fwd")
    return y


_CONV_GN_PARTS = {}   # (conv geometry, groups, rows) -> statistics partials per sample (<= 0: none)


def conv2d_gn(x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor], stride: int, padding: int,
              img_add: Optional[torch.Tensor], groups: int, frames: int, residual: Optional[torch.Tensor] = None):
    """K10 ``conv(x) + img_add[image]`` (the resnet's ``conv1(.) + temb``, resnet.py:146-156: two
    roundings) that also leaves the GroupNorm statistics of its output -- the next norm2's
    (resnet.py:158), ``groups`` groups over ``frames`` consecutive images -- as per-tile (count, mean,
    M2) partials written by the epilogue, so the GroupNorm needs no statistics pass.  ``residual``
    (instead of ``img_add``): ``residual + conv(x)`` (the resnet's output, whose statistics the next
    Transformer3DModel.norm takes, attention.py:110).  Returns
    (y, (partials, parts)), or None when the shape cannot produce them in one pass (split-K, tile /
    group geometry): the caller then runs the conv and the GroupNorm as usual."""
    if not x.is_contiguous(memory_format=torch.channels_last) or x.dtype != torch.bfloat16:
        return None
    w = weight if weight.is_contiguous(memory_format=torch.channels_last) else \
        weight.contiguous(memory_format=torch.channels_last)
    if bias is not None and (bias.dtype != x.dtype or not bias.is_contiguous()):
        bias = bias.to(x.dtype).contiguous()
    a, shape = _conv_args(x, w, bias, None, None, stride, padding)
    N, Cout, Ho, Wo = shape
    if N % frames or (img_add is not None and (tuple(img_add.shape) != (N, Cout) or img_add.dtype != x.dtype)):
        return None
    a.gn_groups, a.gn_rows = groups, frames * Ho * Wo
    lib = _lib.load()
    key = (a.batch, a.in_h, a.in_w, a.cin, a.cout, a.kernel, a.stride, a.pad, groups, frames)
    parts = _CONV_GN_PARTS.get(key)
    if parts is None:
        parts = _CONV_GN_PARTS[key] = int(lib.vp2p_conv2d_gn_parts(ctypes.byref(a)))
    if parts <= 0:
        return None
    y = torch.empty(shape, device=x.device, dtype=x.dtype, memory_format=torch.channels_last)
    partials = torch.empty((N // frames) * parts * groups * 3, device=x.device, dtype=torch.float32)
    if residual is not None:
        if img_add is not None or residual.shape != y.shape or residual.dtype != y.dtype:
            return None
        if not residual.is_contiguous(memory_format=torch.channels_last):
            residual = residual.contiguous(memory_format=torch.channels_last)
        a.residual = _ptr(residual)
    if img_add is not None:
        img_add = img_add.contiguous()
        a.img_add = _ptr(img_add)
    a.y, a.gn_partials = _ptr(y), _ptr(partials)
    check(lib.vp2p_conv2d_fwd(ctypes.byref(a), _stream()), "vp2p_conv2d_fwd(gn)")
    return y, (partials, parts)


def group_norm_from_partials(x: torch.Tensor, num_groups: int, weight: Optional[torch.Tensor],
                             bias: Optional[torch.Tensor], eps: float, frames: int, stats, silu: bool = False,
                             shard=None) -> torch.Tensor:
    """The apply half of ``group_norm`` on statistics its producer left (``conv2d_gn``): the
    partials are merged into {mean, rstd} per (batch, group) -- across the frame shards' ranks
    through the merged-triple exchange -- and one apply launch normalises (+ SiLU)."""
    partials, parts = stats
    out = torch.empty_like(x, memory_format=torch.channels_last)
    a = _gn_args(x, num_groups, weight, bias, eps, frames, silu, None, out)
    lib = _lib.load()
    s = _stream()
    B = x.shape[0] // frames
    st = torch.empty(B * num_groups * 2, device=x.device, dtype=torch.float32)
    if shard is not None and shard.world > 1:
        tri = torch.empty(B * num_groups * 3, device=x.device, dtype=torch.float32)
        check(lib.vp2p_group_norm_merge_parts(ctypes.byref(a), _ptr(partials), parts, _ptr(tri), s),
              "vp2p_group_norm_merge_parts")
        tri = shard.all_gather_flat(tri)
        check(lib.vp2p_group_norm_finalize_merged(ctypes.byref(a), _ptr(tri), shard.world, _ptr(st), s),
              "vp2p_group_norm_finalize_merged")
    elif parts < GN_FINALIZE_MIN_PARTS:       # few partials: every apply block merges them (one launch)
        check(lib.vp2p_group_norm_apply_parts(ctypes.byref(a), _ptr(partials), parts, s), "vp2p_group_norm_apply_parts")
        return out
    else:
        check(lib.vp2p_group_norm_finalize_parts(ctypes.byref(a), _ptr(partials), parts, _ptr(st), s),
              "vp2p_group_norm_finalize_parts")
    check(lib.vp2p_group_norm_apply_stats(ctypes.byref(a), _ptr(st), s), "vp2p_group_norm_apply_stats")
    return out


class ConvSelector:
    """Per-shape choice between a K10 launch and the library path (MIOpen convolution, hipBLASLt
    GEMM + K9 / a separate add).

    The choice is read from an in-tree table (``miopen_db/kernel_choices.json``), measured once on
    the MI355X by ``tools/choose_kernels.py`` for every shape the pipeline, the inversion, the
    null-text loop and the multi-GPU layouts run.  K10 and the library are not bit-equal, so a
    fixed table keeps the numerics identical from run to run, box to box and rank to rank (a
    per-process timing race would not).  Shapes missing from the table take a fixed rule: K10
    wherever it covers the shape.  ``VP2P_CONV``: ``table`` (default) | ``k10`` | ``library`` |
    ``tune`` (time both on first use -- the mode the table is generated in)."""

    TABLE = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                         "miopen_db", "kernel_choices.json")

    def __init__(self):
        self.mode = os.environ.get("VP2P_CONV", "table")
        if self.mode not in ("table", "k10", "library", "tune"):
            raise ValueError(f"VP2P_CONV={self.mode!r}: expected table | k10 | library | tune")
        self.table = {}
        if os.path.exists(self.TABLE):
            with open(self.TABLE) as fh:
                self.table = {k: bool(v) for k, v in json.load(fh)["choices"].items()}
        self.choice = {}
        self._supported = {}

    @staticmethod
    def key_str(key) -> str:
        return "|".join(str(k) for k in key)

    def pick(self, key, supported: bool, k10, library) -> bool:
        if not supported or self.mode == "library":
            return False
        if self.mode == "k10":
            return True
        ks = self.key_str(key)
        use = self.choice.get(ks)
        if use is None:
            use = self._faster(k10, library) if self.mode == "tune" else self.table.get(ks, True)
            self.choice[ks] = use
        return use

    def run(self, x, weight, bias, stride: int, padding: int, residual, library, upsample: bool = False,
            x2: Optional[torch.Tensor] = None):
        """``x2``: the input is torch.cat([x, x2], dim=1); K10 reads the two parts (1x1), ``library``
        must build the cat itself.  The table key is the cat's shape."""
        def k10():
            return conv2d(x, weight, bias, stride, padding, residual=residual, upsample=upsample, x2=x2)

        def lib():
            y = library()
            return y if residual is None else residual + y

        xs = tuple(x.shape) if x2 is None else (x.shape[0], x.shape[1] + x2.shape[1]) + tuple(x.shape[2:])
        key = ("conv", xs, tuple(weight.shape), stride, padding, residual is not None, upsample)
        skey = (key, x2 is not None, x.dtype, weight.dtype, x.is_cuda, x.is_contiguous(memory_format=torch.channels_last),
                x2 is None or x2.is_contiguous(memory_format=torch.channels_last))
        sup = self._supported.get(skey)
        if sup is None:       # a pure function of shapes, dtypes and layouts: asked once per key
            sup = self._supported[skey] = conv2d_supported(x, weight, stride, padding, upsample, x2)
        if self.pick(key, sup, k10, lib):
            return k10()
        return lib()

    def prefers_k10(self, x, weight, stride: int, padding: int, residual: bool = False) -> bool:
        """Whether ``run`` would take K10 for this convolution (no upsample or second source; with
        or without a residual add: the same table key ``run`` builds) -- without running anything
        ("tune" mode: no, it times on first use)."""
        if self.mode == "tune":
            return False
        key = ("conv", tuple(x.shape), tuple(weight.shape), stride, padding, bool(residual), False)
        skey = (key, False, x.dtype, weight.dtype, x.is_cuda, x.is_contiguous(memory_format=torch.channels_last), True)
        sup = self._supported.get(skey)
        if sup is None:
            sup = self._supported[skey] = conv2d_supported(x, weight, stride, padding)
        return self.pick(key, sup, None, None)

    @staticmethod
    def _faster(k10, library) -> bool:
        times = []
        for fn in (k10, library):
            for _ in range(2):
                fn()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(5):
                fn()
            e.record()
            e.synchronize()
            times.append(s.elapsed_time(e))
        return times[0] < times[1]


CONV = ConvSelector()


def geglu_interleave(weight: torch.Tensor, bias: Optional[torch.Tensor]):
    """Row order K10's GEGLU epilogue expects: per 32 rows, 16 value rows then the 16 matching gate
    rows (GEGLU.proj is [value; gate], diffusers' ``chunk(2, dim=-1)``), so that a wave's MFMA output
    tiles 2q and 2q + 1 hold the value and the gate of the same 16 channels in the same lanes."""
    n2, k = weight.shape
    inner = n2 // 2
    if inner % 80:
        raise ValueError("GEGLU inner width must be a multiple of 80")
    t = inner // 16
    w = torch.stack([weight[:inner].reshape(t, 16, k), weight[inner:].reshape(t, 16, k)], 1).reshape(n2, k)
    b = None if bias is None else torch.stack([bias[:inner].reshape(t, 16), bias[inner:].reshape(t, 16)], 1).reshape(n2)
    return w.contiguous(), (None if b is None else b.contiguous())


def linear_geglu_supported(x: torch.Tensor, weight: torch.Tensor) -> bool:
    if x.dtype != torch.bfloat16 or weight.dtype != torch.bfloat16 or not x.is_cuda or not x.is_contiguous():
        return False
    M = x.numel() // x.shape[-1]
    a = _lib.ConvArgs(None, None, None, None, None, 1, M, 1, x.shape[-1], weight.shape[0], M, 1, 1, 1, 0,
                      _lib.BF16, _lib.CONV_EPI_GEGLU)
    return weight.shape[0] % 160 == 0 and bool(_lib.load().vp2p_conv2d_supported(ctypes.byref(a)))


def linear_geglu(x: torch.Tensor, w_il: torch.Tensor, b_il: Optional[torch.Tensor]) -> torch.Tensor:
    """GEGLU(x) = value * gelu(gate) with (value, gate) = x @ W^T + b, in one K10 launch (the
    projection's (M, 2*inner) output is never written).  ``w_il``/``b_il`` from ``geglu_interleave``."""
    K = x.shape[-1]
    M = x.numel() // K
    n2 = w_il.shape[0]
    y = torch.empty(*x.shape[:-1], n2 // 2, device=x.device, dtype=x.dtype)
    a = _lib.ConvArgs(_ptr(x), _ptr(w_il), _ptr(b_il), None, _ptr(y), 1, M, 1, K, n2, M, 1, 1, 1, 0,
                      _lib.BF16, _lib.CONV_EPI_GEGLU)
    check(_lib.load().vp2p_conv2d_fwd(ctypes.byref(a), _stream()), "vp2p_conv2d_fwd(geglu)")
    return y


def linear_residual(x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor],
                    residual: torch.Tensor) -> torch.Tensor:
    """residual + x @ W^T + b on K10's GEMM core (a 1x1 convolution over M = rows pixels), the add
    fused into the epilogue.  x: (..., K) contiguous bf16; residual: (..., N) contiguous."""
    K = x.shape[-1]
    M = x.numel() // K
    N = weight.shape[0]
    y = torch.empty(*x.shape[:-1], N, device=x.device, dtype=x.dtype)
    a = _lib.ConvArgs(_ptr(x), _ptr(weight), _ptr(bias), _ptr(residual), _ptr(y), 1, M, 1, K, N, M, 1, 1, 1, 0,
                      _lib.BF16, _lib.CONV_EPI_NONE)
    lib = _lib.load()
    ws = None
    wsb = lib.vp2p_conv2d_workspace_bytes(ctypes.byref(a))
    if wsb > 0:
        ws = torch.empty(wsb // 4, device=x.device, dtype=torch.float32)
        a.workspace = _ptr(ws)
    check(lib.vp2p_conv2d_fwd(ctypes.byref(a), _stream()), "vp2p_conv2d_fwd(linear)")
    return y


class LinearRule:
    """Which plain projections run on K10's GEMM core instead of hipBLASLt: per (K, N), the ranges of
    row counts M over which K10 measured faster (``linear_rules`` in the in-tree
    ``miopen_db/kernel_choices.json``, written by ``tools/linear_choose.py`` on the MI355X from
    profiles/r03_linear_choose.jsonl).  A range [lo, hi] covers the measured M between lo and hi; a
    range that starts at the smallest measured M extends down to 0 and one that ends at the largest
    extends up without bound.  A fixed table, so the kernel (and the numerics: K10 and hipBLASLt are
    not bit-equal at every shape) is the same on every run, box and rank; pairs missing from it stay on
    hipBLASLt.  ``VP2P_LINEAR``: ``table`` (default) | ``k10`` | ``library`` -- A/B, read once."""

    DEFAULT = {"320|320": [[65536, None]], "320|640": [[65536, None]]}   # round 2's rule, no table

    def __init__(self):
        self.mode = os.environ.get("VP2P_LINEAR", "table")
        if self.mode not in ("table", "k10", "library"):
            raise ValueError(f"VP2P_LINEAR={self.mode!r}: expected table | k10 | library")
        self.rules = dict(self.DEFAULT)
        if os.path.exists(ConvSelector.TABLE):
            with open(ConvSelector.TABLE) as fh:
                table = json.load(fh).get("linear_rules")
            if table is not None:
                self.rules = {k: [list(r) for r in v] for k, v in table.items()}

    def use_k10(self, M: int, K: int, N: int) -> bool:
        if self.mode != "table":
            return self.mode == "k10"
        for lo, hi in self.rules.get(f"{K}|{N}", ()):
            if (lo is None or M >= lo) and (hi is None or M <= hi):
                return True
        return False


LINEAR = LinearRule()


def linear_k10_ok(x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor]) -> bool:
    """K10's GEMM core takes x @ W^T (+ b): bf16, contiguous, K % 64 == 0, N % 160 == 0, no autograd."""
    return (x.dtype == torch.bfloat16 and weight.dtype == torch.bfloat16 and x.is_cuda and x.dim() >= 2
            and not torch.is_grad_enabled() and x.is_contiguous() and weight.is_contiguous()
            and (bias is None or (bias.dtype == x.dtype and bias.is_contiguous()))
            and x.shape[-1] % 64 == 0 and weight.shape[0] % 160 == 0 and x.numel() > 0)


def linear_k10(x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor] = None,
               alpha: float = 1.0) -> torch.Tensor:
    """alpha * (x @ W^T + b) on K10's GEMM core (a 1x1 convolution over M = rows pixels), one rounding."""
    K, N = x.shape[-1], weight.shape[0]
    M = x.numel() // K
    y = torch.empty(*x.shape[:-1], N, device=x.device, dtype=x.dtype)
    a = _lib.ConvArgs(_ptr(x), _ptr(weight), _ptr(bias), None, _ptr(y), 1, M, 1, K, N, M, 1, 1, 1, 0,
                      _lib.BF16, _lib.CONV_EPI_NONE)
    a.alpha = float(alpha)
    lib = _lib.load()
    ws = None
    wsb = lib.vp2p_conv2d_workspace_bytes(ctypes.byref(a))
    if wsb > 0:
        ws = torch.empty(wsb // 4, device=x.device, dtype=torch.float32)
        a.workspace = _ptr(ws)
    check(lib.vp2p_conv2d_fwd(ctypes.byref(a), _stream()), "vp2p_conv2d_fwd(linear)")
    return y


def linear_add(x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor],
               residual: torch.Tensor) -> torch.Tensor:
    """residual + (x @ W^T + b) with the reference's two roundings (the projection, then the sum):
    one K10 launch with the add in its epilogue where ``LINEAR`` puts the projection on K10,
    otherwise the projection (``linear``) and a separate add."""
    K, N = x.shape[-1], weight.shape[0]
    M = x.numel() // max(K, 1)
    if (linear_k10_ok(x, weight, bias) and LINEAR.use_k10(M, K, N) and residual.is_contiguous()
            and residual.dtype == x.dtype and residual.shape[:-1] == x.shape[:-1] and residual.shape[-1] == N):
        return linear_residual(x, weight, bias, residual)
    return linear(x, weight, bias) + residual


def linear_add_fused(M: int, K: int, N: int) -> bool:
    """Whether ``linear_add`` runs as one K10 launch for this shape (a fixed table lookup)."""
    return LINEAR.use_k10(M, K, N) and K % 64 == 0 and N % 160 == 0


_WT = {}       # (weight storage, version, shape) -> contiguous W^T (frozen weights: the backward's GEMM operand)


def transposed_weight(w: torch.Tensor) -> torch.Tensor:
    """W^T, contiguous, cached while the weight is unchanged (the key holds the weight's version; the
    entry holds the weight, so its memory cannot be recycled under the key)."""
    key = (version_key(w), tuple(w.shape), w.dtype)
    hit = _WT.get(key) if key[0] is not None else None
    if hit is None:
        with torch.no_grad():
            hit = (w, w.detach().t().contiguous())
        if key[0] is not None:
            _WT[key] = hit
    return hit[1]


def _kernel_flipped(w: torch.Tensor) -> torch.Tensor:
    """The transposed convolution's kernel as a forward one: w'[ci, co, i, j] = w[co, ci, k-1-i, k-1-j]
    (channels-last), cached like ``transposed_weight``."""
    key = ("conv_t", version_key(w), tuple(w.shape), w.dtype)
    hit = _WT.get(key) if key[1] is not None else None
    if hit is None:
        with torch.no_grad():
            hit = (w, w.detach().flip(2, 3).transpose(0, 1).contiguous(memory_format=torch.channels_last))
        if key[1] is not None:
            _WT[key] = hit
    return hit[1]


def conv2d_input_grad(in_shape, weight: torch.Tensor, dy: torch.Tensor, stride: int, padding: int) -> torch.Tensor:
    """dL/dx of a 2-D convolution with a frozen ``weight``, for the input shape ``in_shape``.  Stride 1
    with 'same' padding (the 3x3 and 1x1 InflatedConv3d of the resnets, transformers and up blocks) is
    itself a forward convolution of dy with the flipped, transposed kernel -- run on K10 where it
    covers the shape (bf16, channel counts); strided ones (Downsample3D) and the rest take MIOpen's
    backward-data."""
    k = weight.shape[-1]
    if stride == 1 and 2 * padding == k - 1 and dy.dtype == torch.bfloat16 and dy.is_cuda:
        dyc = dy.contiguous(memory_format=torch.channels_last)
        wt = _kernel_flipped(weight)
        if conv2d_supported(dyc, wt, 1, padding):
            return conv2d(dyc, wt, None, 1, padding)
    return torch.nn.grad.conv2d_input(tuple(in_shape), weight, dy, stride, padding)


def linear(x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor] = None,
           alpha: Optional[float] = None) -> torch.Tensor:
    """nn.Linear (``alpha``: alpha * (x @ W^T + b), one rounding -- the pre-scaled FrameAttention query).
    K10's GEMM core where ``LINEAR`` says it is faster for the shape, hipBLASLt elsewhere.  Under
    autograd with frozen weights (the null-text loop) the same dispatch runs forward and backward
    (``autograd.FrozenLinear``); trainable weights differentiate through torch."""
    if (alpha is None and torch.is_grad_enabled() and x.requires_grad and x.dtype == torch.bfloat16
            and not weight.requires_grad and (bias is None or not bias.requires_grad)):
        from .autograd import FrozenLinear
        return FrozenLinear.apply(x, weight, bias)
    K, N = x.shape[-1], weight.shape[0]
    M = x.numel() // max(K, 1)
    if linear_k10_ok(x, weight, bias) and LINEAR.use_k10(M, K, N):
        return linear_k10(x, weight, bias, 1.0 if alpha is None else alpha)
    if alpha is None:
        return F.linear(x, weight, bias)
    # one library GEMM with alpha and beta in its epilogue
    x2 = x.reshape(-1, K)
    if bias is None:
        y = torch.addmm(x2.new_zeros(()), x2, weight.t(), beta=0, alpha=alpha)
    else:
        y = torch.addmm(bias, x2, weight.t(), beta=alpha, alpha=alpha)
    return y.view(*x.shape[:-1], N)


def linear_residual_supported(x: torch.Tensor, weight: torch.Tensor, residual: torch.Tensor) -> bool:
    if x.dtype != torch.bfloat16 or weight.dtype != torch.bfloat16 or not x.is_cuda:
        return False
    if not (x.is_contiguous() and weight.is_contiguous() and residual.is_contiguous()):
        return False
    K = x.shape[-1]
    M = x.numel() // K
    a = _lib.ConvArgs(None, None, None, None, None, 1, M, 1, K, weight.shape[0], M, 1, 1, 1, 0,
                      _lib.BF16, _lib.CONV_EPI_NONE)
    return bool(_lib.load().vp2p_conv2d_supported(ctypes.byref(a)))
