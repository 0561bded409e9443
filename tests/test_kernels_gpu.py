"""Kernel parity on the MI355X: every HIP kernel vs the CPU oracle on the same inputs.

Tolerances (BASELINE.json north_star): fp32 <= 1e-4 relative, bf16 <= 2e-2 relative (measured
as max|err| / max|ref|).  The reference's hooked softmax uses one global max (ptp_utils.py:217);
the kernels use a per-row max, equal wherever the reference does not underflow -- each test
asserts the oracle output is finite (no underflowed rows) before comparing.
"""
import numpy as np
import pytest
import torch

from oracle import p2p_oracle as O

pytestmark = pytest.mark.gpu

DEV = "cuda"
TOL = {torch.float32: 1e-4, torch.bfloat16: 2e-2}


def _rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


def _rand(shape, seed, scale=1.0, dtype=torch.float32):
    g = np.random.default_rng(seed)
    x = torch.from_numpy((g.standard_normal(shape) * scale).astype(np.float32)).to(dtype)
    return x  # CPU; values already rounded to dtype


def _np(t):
    return t.float().cpu().numpy()


@pytest.fixture(scope="module", autouse=True)
def _lib():
    from vp2p import _lib
    _lib.load()
    assert torch.cuda.is_available()


# ------------------------------------------------------------------------------------------------
def _prescale(q, d):
    """q' = q * d**-0.5 * log2(e) rounded once to q's dtype (what the to_q GEMM's alpha produces), and
    the float64 query the oracle must see for it (q' / c): the oracle then scores exactly q'.k."""
    from vp2p import ops
    c = ops.frame_query_scale(d)
    qs = (q.double() * c).to(q.dtype)
    return qs, (qs.double() / c).numpy()


@pytest.mark.parametrize("prescaled", [False, True])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("d,frames,n", [(40, 3, 200), (80, 2, 256), (160, 2, 144), (40, 8, 64), (40, 2, 300),
                                         (40, 2, 128), (40, 2, 256), (80, 3, 200), (160, 2, 256), (160, 3, 64)])
def test_frame_attention(dtype, d, frames, n, prescaled):
    """Both query conventions: plain q (scale applied in the kernel) and q pre-multiplied by
    scale*log2(e) (the production call, FrameAttention.forward; at d = 40 bf16 it selects the
    folded-max kernel, whose ragged 128-key tiles n = 200 / 64 / 300 exercise; n = 256, a multiple
    of the pp kernel's 256-key tile, takes the res-64 pp kernel as a single tile, n = 128 the x2f
    kernel: several pp tiles are test_frame_attention_pp_tiles; d = 80 / 160: x2f / one-set)."""
    from vp2p import ops
    heads, B = 8, 2
    C = heads * d
    q = _rand((B * frames, n, C), 1, 1.0, dtype)
    k = _rand((B * frames, n, C), 2, 1.0, dtype)
    v = _rand((B * frames, n, C), 3, 1.0, dtype)
    qref = _np(q)
    if prescaled:
        q, qref = _prescale(q, d)
    ref = O.frame_attention(qref, _np(k), _np(v), frames, heads)
    out = ops.frame_attention(q.to(DEV), k.to(DEV), v.to(DEV), frames, heads, q_prescaled=prescaled)
    torch.cuda.synchronize()
    assert _rel(_np(out), ref) < TOL[dtype], _rel(_np(out), ref)
    # frame-0-only K/V (the production call) must give the identical result
    k0 = k.reshape(B, frames, n, C)[:, 0].contiguous().to(DEV)
    v0 = v.reshape(B, frames, n, C)[:, 0].contiguous().to(DEV)
    out0 = ops.frame_attention(q.to(DEV), k0, v0, frames, heads, q_prescaled=prescaled)
    torch.cuda.synchronize()
    assert torch.equal(out0, out)


@pytest.mark.parametrize("d,n,spikes", [(40, 1024, (300, 900)), (40, 4096, (300, 1380)), (40, 4096, ()),
                                         (80, 1024, (300, 700)), (80, 2048, (200, 1500)), (80, 128, ()),
                                         (160, 256, (70, 200)), (160, 1024, (100, 700)), (160, 64, (20,))])
def test_frame_attention_pp_tiles(d, n, spikes):
    """The UNet's bf16 pre-scaled call over many key tiles: d = 40 is the pipelined kernel
    (frame_attn_pp.hip, 256-key tiles: 4 and 16 tiles, its 3-slot LDS ring wraps -- tile t + 2 lands
    in tile t - 1's slot -- and its XOR-swizzled image is read at every block offset); d = 80 / 160
    the x2f / one-set kernels at the res-32 / res-16 / res-8 key counts and beyond.  Spike keys in an
    early and a later tile make the running max move part-way through the key axis (the pp kernel's
    row-sum growth check every 512 keys rescales its in-flight P and S).  float64 oracle on the same
    bf16 inputs, 2e-2 of max|ref|, plus the lse."""
    from vp2p import ops
    heads, B, frames = 2, 1, 2
    C = heads * d
    q = _rand((B * frames, n, C), 11, 1.0)
    k = _rand((B, n, C), 12, 1.0)
    for i, key in enumerate(spikes):
        k[0, key] *= 6.0 + 4.0 * i
    v = _rand((B, n, C), 13, 1.0)
    q, k, v = (x.to(torch.bfloat16) for x in (q, k, v))
    q, qref = _prescale(q, d)
    ref = O.frame_attention(qref, _np(k), _np(v), frames, heads)
    assert np.isfinite(ref).all()
    lse = torch.empty(B * heads, frames * n, device=DEV)
    out = ops.frame_attention(q.to(DEV), k.to(DEV), v.to(DEV), frames, heads, lse=lse, q_prescaled=True)
    torch.cuda.synchronize()
    assert _rel(_np(out), ref) < 2e-2, _rel(_np(out), ref)
    qd = np.asarray(qref, np.float64).reshape(B, frames * n, heads, d).transpose(0, 2, 1, 3)
    kd = _np(k).astype(np.float64).reshape(B, n, heads, d).transpose(0, 2, 1, 3)
    sc = qd @ kd.transpose(0, 1, 3, 2) * d ** -0.5 * np.log2(np.e)
    mx = sc.max(-1, keepdims=True)
    lse_ref = (mx[..., 0] + np.log2(np.exp2(sc - mx).sum(-1))).reshape(B * heads, frames * n)
    assert np.abs(lse.cpu().numpy() - lse_ref).max() < 5e-2


def test_frame_attention_large_logits():
    """Force the online-softmax rescale branch: a spike key late in the sequence (rule 26)."""
    from vp2p import ops
    heads, B, frames, n, d = 8, 1, 2, 512, 40
    C = heads * d
    q = _rand((B * frames, n, C), 4, 1.0)
    k = _rand((B * frames, n, C), 5, 1.0)
    k[0, 450] *= 12.0
    v = _rand((B * frames, n, C), 6, 1.0)
    ref = O.frame_attention(_np(q), _np(k), _np(v), frames, heads)
    out = ops.frame_attention(q.to(DEV), k.to(DEV), v.to(DEV), frames, heads)
    torch.cuda.synchronize()
    assert _rel(_np(out), ref) < 1e-4


@pytest.mark.parametrize("d", [40, 80, 160])
@pytest.mark.parametrize("prescaled", [False, True])
@pytest.mark.parametrize("spike", [4.0, 12.0, "overflow", "overflow_v"])
def test_frame_attention_bf16_spikes(spike, prescaled, d):
    """bf16 (d = 40: the x2f kernel; d = 80: x2f; d = 160: one-set): a late key whose logits jump far
    above the first block's max.
    4x / 12x exercise the row-sum rescale; "overflow" aligns the key with one query so that its logit
    is ~100 nats above the running max (p would overflow bf16/fp32), forcing the exact per-row
    fallback; "overflow_v" puts the logit ~80 nats up (p ~ 2^114, the row sum stays finite) on a
    value row of magnitude 2^20, so only the O accumulator overflows -- the fallback must catch that
    too.  Tolerance: the bf16 bar of the north star, 2e-2 of max|ref|."""
    from vp2p import ops
    heads, B, frames, n = 8, 1, 2, 512
    C = heads * d
    q = _rand((B * frames, n, C), 4, 1.0)
    k = _rand((B * frames, n, C), 5, 1.0)
    if spike == "overflow":
        k[0, 450, :d] = 16.0 * q[1, 100, :d]
        k[0, 300, d:2 * d] = 12.0 * q[0, 7, d:2 * d]
    elif spike == "overflow_v":      # logit of query (1, 100) on key 450: 80 nats (p ~ 2^115)
        qq = float((q[1, 100, :d].double() ** 2).sum())
        k[0, 450, :d] = (80.0 * d ** 0.5 / qq) * q[1, 100, :d]
    else:
        k[0, 450] *= spike
    v = _rand((B * frames, n, C), 6, 1.0)
    if spike == "overflow_v":
        v[0, 450, :d] *= 2.0 ** 20
    q, k, v = (x.to(torch.bfloat16) for x in (q, k, v))
    qref = _np(q)
    if prescaled:   # the folded-max kernel: its growth rescale, m moves and overflow fallback
        q, qref = _prescale(q, d)
    ref = O.frame_attention(qref, _np(k), _np(v), frames, heads)
    assert np.isfinite(ref).all()
    out = ops.frame_attention(q.to(DEV), k.to(DEV), v.to(DEV), frames, heads, q_prescaled=prescaled)
    lse = torch.empty(B * heads, frames * n, device=DEV)
    out2 = ops.frame_attention(q.to(DEV), k.to(DEV), v.to(DEV), frames, heads, lse=lse, q_prescaled=prescaled)
    torch.cuda.synchronize()
    assert torch.isfinite(out.float()).all()
    assert _rel(_np(out), ref) < 2e-2, _rel(_np(out), ref)
    assert torch.equal(out, out2)
    # log-sum-exp (log2 units, scale folded in) against float64
    qd = np.asarray(qref, np.float64).reshape(B, frames * n, heads, d).transpose(0, 2, 1, 3)
    kd = _np(k).astype(np.float64).reshape(B, frames, n, heads, d)[:, 0].transpose(0, 2, 1, 3)
    sc = qd @ kd.transpose(0, 1, 3, 2) * d ** -0.5 * np.log2(np.e)
    mx = sc.max(-1, keepdims=True)
    lse_ref = (mx[..., 0] + np.log2(np.exp2(sc - mx).sum(-1))).reshape(B * heads, frames * n)
    assert np.abs(lse.cpu().numpy() - lse_ref).max() < 5e-2


# ------------------------------------------------------------------------------------------------
def _controller(tokenizer, name, step):
    import spec
    prompts, swap, blend, eq, cross, self_ = spec.CONFIGS[name]
    ctrl = O.EditController(prompts, swap, {"default_": cross}, self_, tokenizer,
                            blend_words=None if blend is None else ((blend[0],), (blend[1],)),
                            eq_params=eq)
    ctrl.cur_step = step
    return ctrl


def _plan(ctrl, lb_alpha=None):
    from vp2p import _lib, ops
    mode = _lib.EDIT_REPLACE if ctrl.is_replace else _lib.EDIT_REFINE
    return ops.CrossEditPlan(
        ctrl.batch_size, mode, ctrl.equalizer is not None, torch.from_numpy(ctrl.cross_replace_alpha),
        mapper=ctrl.mapper, refine_alpha=None if ctrl.is_replace else ctrl.alphas.reshape(ctrl.batch_size - 1, -1),
        equalizer=ctrl.equalizer, lb_word_alpha=lb_alpha)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("name,step,d", [("rabbit", 0, 40), ("rabbit", 12, 40), ("car", 3, 40), ("man", 5, 40),
                                         ("bird", 30, 40), ("rabbit", 12, 160), ("bird", 30, 80), ("car", 20, 160)])
def test_cross_attention_p2p(tokenizer, dtype, name, step, d):
    """Edit launches (inside the cross-replace window) and non-edit launches (K2 v3: K/V in LDS) at
    the UNet's head dims, with LocalBlend sums and stored maps."""
    from vp2p import ops
    heads, P, frames, n = 8, 2, 2, 256
    B, C = 2 * P, heads * d
    ctrl = _controller(tokenizer, name, step)
    lb_alpha = ctrl.local_blend.alpha_layers.reshape(P, 77) if ctrl.local_blend else np.ones((P, 77), np.float32)
    q = _rand((B * frames, n, C), 7, 1.0, dtype)
    k = _rand((B, 77, C), 8, 1.0, dtype)
    v = _rand((B, 77, C), 9, 1.0, dtype)
    kf = np.repeat(_np(k), frames, axis=0)   # context repeated per frame (attention.py:95)
    vf = np.repeat(_np(v), frames, axis=0)
    ref_out, ref_p = O.controlled_core(_np(q), kf, vf, heads, True, ctrl, "up")
    assert np.isfinite(ref_p).all() and np.isfinite(ref_out).all()
    plan = _plan(ctrl, lb_alpha)
    lb_acc = torch.zeros(P, frames, n, device=DEV)
    probs = torch.empty(B * frames * heads, n, 77, device=DEV)
    # the flag the fused protocol passes (controllers.fused_begin): edit launches only inside the
    # cross-replace window (outside it the reference edits nothing, Reweight included)
    edit = bool(ctrl.cross_replace_alpha.reshape(ctrl.cross_replace_alpha.shape[0], -1)[step].max() > 0)
    out = ops.cross_attention_p2p(q.to(DEV), k.to(DEV), v.to(DEV), frames, heads, plan=plan, step=step,
                                  edit=edit, lb_acc=lb_acc, probs_out=probs)
    torch.cuda.synchronize()
    tol = TOL[dtype]
    assert _rel(probs.cpu().numpy(), ref_p) < tol, _rel(probs.cpu().numpy(), ref_p)
    assert _rel(_np(out), ref_out) < tol, _rel(_np(out), ref_out)
    cond = ref_p.reshape(B, frames, heads, n, 77)[P:]
    ref_lb = np.einsum("pfhnw,pw->pfn", cond, lb_alpha)
    assert _rel(lb_acc.cpu().numpy(), ref_lb) < tol


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("d", [40, 80, 160])
def test_cross_attention_plain(dtype, d):
    """No controller: plain hooked softmax-attention (DummyController, ptp_utils.py:225-234)."""
    from vp2p import ops
    heads, frames, n, B = 8, 3, 100, 3
    C = heads * d
    q = _rand((B * frames, n, C), 10, 1.0, dtype)
    k = _rand((B, 77, C), 11, 1.0, dtype)
    v = _rand((B, 77, C), 12, 1.0, dtype)
    ref, _ = O.controlled_core(_np(q), np.repeat(_np(k), frames, 0), np.repeat(_np(v), frames, 0),
                               heads, True, None)
    out = ops.cross_attention_p2p(q.to(DEV), k.to(DEV), v.to(DEV), frames, heads)
    torch.cuda.synchronize()
    assert _rel(_np(out), ref) < TOL[dtype]


# ------------------------------------------------------------------------------------------------
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("frames,d,step", [(8, 40, 0), (8, 40, 30), (24, 80, 3), (3, 160, 1), (16, 40, 0),
                                           (48, 40, 0), (128, 80, 3), (64, 160, 1), (33, 32, 30)])
def test_temporal_attention_p2p(tokenizer, dtype, frames, d, step):
    from vp2p import ops
    heads, P, n = 8, 2, 48
    B, C = 2 * P, heads * d
    ctrl = _controller(tokenizer, "rabbit", step)
    # '(b f) n c' inputs; the oracle consumes the reference's '(b d) f c' rearrangement
    q = _rand((B * frames, n, C), 13, 1.0, dtype)
    k = _rand((B * frames, n, C), 14, 1.0, dtype)
    v = _rand((B * frames, n, C), 15, 1.0, dtype)
    to_bd = lambda t: _np(t).reshape(B, frames, n, C).transpose(0, 2, 1, 3).reshape(B * n, frames, C)  # noqa
    ref_out, ref_p = O.controlled_core(to_bd(q), to_bd(k), to_bd(v), heads, False, ctrl, "down")
    assert np.isfinite(ref_out).all()
    replace = ctrl.num_self_replace[0] <= step < ctrl.num_self_replace[1]
    probs = torch.empty(B * n * heads, frames, frames, device=DEV)
    out = ops.temporal_attention_p2p(q.to(DEV), k.to(DEV), v.to(DEV), frames, heads, prompts=P,
                                     self_replace=replace, probs_out=probs)
    torch.cuda.synchronize()
    got = _np(out).reshape(B, frames, n, C).transpose(0, 2, 1, 3).reshape(B * n, frames, C)
    assert _rel(probs.cpu().numpy(), ref_p) < TOL[dtype]
    assert _rel(got, ref_out) < TOL[dtype], _rel(got, ref_out)
    # the reference '(b d)' layout through the strided entry point gives the same numbers
    bd = lambda t: torch.from_numpy(to_bd(t)).to(dtype).to(DEV)  # noqa
    out_bd = ops.temporal_attention_p2p_bd(bd(q), bd(k), bd(v), B, heads, prompts=P, self_replace=replace)
    torch.cuda.synchronize()
    assert torch.equal(out_bd.cpu().float(), torch.from_numpy(got))


@pytest.mark.parametrize("mode,n", [("edit", 4096), ("replace", 4096), ("cond_only", 4096), ("plain2", 4096),
                                    ("replace", 4100), ("plain4", 2050)])
def test_temporal_stream(tokenizer, mode, n):
    """K3s, the persistent res-64 stream (bf16, d 40, 8 frames, q|k|v slices of one projection as the
    UNet calls it): the same numbers as the short kernel (VP2P_K3_STREAM=0), and the oracle on the
    P2P cases -- edit / self-replace / the CFG-split conditional half / plain row pairs, and ragged
    item counts (tokens 4100, 2050) that leave the persistent grid's last round partial."""
    import os
    from vp2p import ops
    heads, d, frames = 8, 40, 8
    C = heads * d
    P = 2
    B = {"edit": 4, "replace": 4, "cond_only": 2, "plain2": 2, "plain4": 4}[mode]
    g = torch.Generator().manual_seed(77)
    qkv = (torch.randn(B * frames, n, 3 * C, generator=g) * 2.0).to(torch.bfloat16).to(DEV)
    q, k, v = qkv[..., :C], qkv[..., C:2 * C], qkv[..., 2 * C:]
    kw = {}
    if mode in ("edit", "replace", "cond_only"):
        kw = dict(prompts=P, self_replace=mode != "edit", cond_only=mode == "cond_only")

    def run(stream):
        old = os.environ.get("VP2P_K3_STREAM")
        os.environ["VP2P_K3_STREAM"] = "1" if stream else "0"
        try:
            out = ops.temporal_attention_p2p(q, k, v, frames, heads, **kw)
            torch.cuda.synchronize()
        finally:
            if old is None:
                del os.environ["VP2P_K3_STREAM"]
            else:
                os.environ["VP2P_K3_STREAM"] = old
        return out.float().cpu()
    got, short = run(True), run(False)
    # same MFMAs / softmax roundings; only the zero-padded key positions inside a 16-key MFMA step
    # differ between the two packings, so allow the last bit
    diff = (got - short).abs().max().item()
    assert diff <= 2 ** -7 * short.abs().max().item(), diff
    if mode in ("edit", "replace", "cond_only"):
        ctrl = _controller(tokenizer, "rabbit", 30 if mode == "edit" else 0)
        nt = 64                                   # the oracle on the first 64 tokens
        sub = lambda t: t[:, :nt].float().cpu().numpy().reshape(B, frames, nt, C).transpose(0, 2, 1, 3).reshape(B * nt, frames, C)  # noqa
        if mode == "cond_only":
            # the conditional half alone: the oracle runs the whole [uncond, cond] batch
            full = lambda t: np.concatenate([sub(t), sub(t)])                                             # noqa
            ref, _ = O.controlled_core(full(q), full(k), full(v), heads, False, ctrl, "down")
            ref = ref[B * nt:]
        else:
            ref, _ = O.controlled_core(sub(q), sub(k), sub(v), heads, False, ctrl, "down")
        g2 = got[:, :nt].numpy().reshape(B, frames, nt, C).transpose(0, 2, 1, 3).reshape(B * nt, frames, C)
        assert _rel(g2, ref) < TOL[torch.bfloat16], _rel(g2, ref)


# ------------------------------------------------------------------------------------------------
@pytest.mark.parametrize("t,fast,blend", [(981, True, True), (501, False, True), (21, True, False),
                                          (501, True, "substruct")])
def test_step_fused(t, fast, blend):
    from vp2p import ops
    P, C, F, H, W = 2, 4, 3, 64, 64
    g = np.random.default_rng(20 + t)
    noise = g.standard_normal((2 * P, C, F, H, W)).astype(np.float32)
    lat = g.standard_normal((P, C, F, H, W)).astype(np.float32)
    acc = np.abs(g.standard_normal((P, F, 256))).astype(np.float32) * 5
    if blend == "substruct":     # (sets, P, F, 256): blend words, substruct words (th[1] = 0.5, no pool)
        acc = np.stack([acc, np.abs(g.standard_normal((P, F, 256))).astype(np.float32) * 5])
    d = O.DDIM()
    d.set_timesteps(50)
    eps = O.cfg(noise, 7.5, fast)
    prev = d.step(eps, t, lat)
    if blend:
        lb = O.LocalBlend.__new__(O.LocalBlend)
        lb.th, lb.latent_hw = (0.3, 0.5), (H, W)
        a0 = acc[0] if blend == "substruct" else acc
        mask = lb.mask_from_word_maps((a0 / np.float32(40)).reshape(P, F, 16, 16), True)
        if blend == "substruct":
            mask = mask & ~lb.mask_from_word_maps((acc[1] / np.float32(40)).reshape(P, F, 16, 16), False)
        ref = O.blend_latents(prev, mask)
    else:
        ref = prev
    prev_t = t - 20
    a_t = d.alphas_cumprod[t]
    a_p = d.alphas_cumprod[prev_t] if prev_t >= 0 else d.final_alpha_cumprod
    consts = (np.sqrt(np.float32(1) - a_t), np.sqrt(a_t), np.sqrt(np.float32(1) - a_p - np.float32(0)), np.sqrt(a_p))
    out = ops.step_fused(torch.from_numpy(noise).to(DEV), torch.from_numpy(lat).to(DEV), consts, 7.5, True, fast,
                         lb_acc=torch.from_numpy(acc).to(DEV) if blend else None, lb_count=40.0, lb_th=0.3,
                         lb_sub_th=0.5)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out.cpu().numpy(), ref)


def test_step_fused_inplace_and_nocfg():
    from vp2p import ops
    P, C, F, H, W = 1, 4, 2, 32, 32
    g = np.random.default_rng(99)
    noise = g.standard_normal((P, C, F, H, W)).astype(np.float32)
    lat = g.standard_normal((P, C, F, H, W)).astype(np.float32)
    d = O.DDIM()
    d.set_timesteps(50)
    ref = d.next_step(noise, 21, lat)
    cur, nxt = 1, 21
    consts = (np.sqrt(np.float32(1) - d.alphas_cumprod[cur]), np.sqrt(d.alphas_cumprod[cur]),
              np.sqrt(np.float32(1) - d.alphas_cumprod[nxt]), np.sqrt(d.alphas_cumprod[nxt]))
    x = torch.from_numpy(lat).to(DEV)
    ops.step_fused(torch.from_numpy(noise).to(DEV), x, consts, cfg=False, out=x)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(x.cpu().numpy(), ref)
