"""Whole-network parity: vp2p UNet3D on the MI355X (HIP attention kernels, fused P2P controller)
vs the CPU oracle UNet (oracle/unet_ref.py + oracle controller) on the same weights and inputs.

Small-channel SD-style config (channels 256/256/512/512, 8 heads -> head dims 32/64) so the CPU
side runs in seconds; 64x64 latents so the LocalBlend layers are 16x16 as in the reference.
Weights use std 0.05 and attn_temp.to_out is non-zero (SURVEY finding 10).
"""
import numpy as np
import pytest
import torch

import spec
from oracle import p2p_oracle as O
from oracle import unet_ref

pytestmark = pytest.mark.gpu

CFG = dict(block_out_channels=(256, 256, 512, 512), cross_attention_dim=64, attention_head_dim=8)
F_, P = 2, 2


def _setup(tokenizer, name, dtype, seed=0):
    import vp2p
    from vp2p.unet3d import UNet3DConditionModel, init_random_
    prompts, swap, blend, eq, cross, self_ = spec.CONFIGS[name]
    unet = init_random_(UNet3DConditionModel(**CFG), seed=seed, std=0.05)
    sd = {k: v.clone() for k, v in unet.state_dict().items()}
    unet = unet.to("cuda", dtype).to(memory_format=torch.channels_last)
    ctrl = vp2p.make_controller(prompts, swap, {"default_": cross}, self_, ((blend[0],), (blend[1],)), eq,
                                tokenizer=tokenizer)
    vp2p.register_attention_control(type("M", (), {"unet": unet})(), ctrl)
    octrl = O.EditController(prompts, swap, {"default_": cross}, self_, tokenizer,
                             blend_words=((blend[0],), (blend[1],)), eq_params=eq)
    return unet, sd, ctrl, octrl


def _inputs(seed):
    g = np.random.default_rng(seed)
    x = torch.from_numpy(g.standard_normal((2 * P, 4, F_, 64, 64)).astype(np.float32))
    ctx = torch.from_numpy(g.standard_normal((2 * P, 77, 64)).astype(np.float32))
    ctx[:P] = ctx[0]
    return x, ctx


def _rel(a, b):
    return float((a - b).abs().max() / b.abs().max())


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 2e-4), (torch.bfloat16, 6e-2)])
@pytest.mark.parametrize("name,step", [("rabbit", 0), ("car", 11), ("rabbit", 30)])
def test_unet_forward_matches_oracle(tokenizer, dtype, tol, name, step):
    unet, sd, ctrl, octrl = _setup(tokenizer, name, dtype)
    x, ctx = _inputs(step)
    ctrl.cur_step = octrl.cur_step = step
    with torch.no_grad():
        got = unet(x.cuda().to(dtype), 981 - 20 * step, ctx.cuda().to(dtype)).sample.float().cpu()
    ref = unet_ref.unet_forward(sd, x, 981 - 20 * step, ctx, octrl)
    assert torch.isfinite(ref).all()
    assert _rel(got, ref) < tol, _rel(got, ref)
    assert ctrl.cur_step == octrl.cur_step == step + 1 and ctrl.cur_att_layer == 0
    # LocalBlend reduction: kernel-accumulated sum vs the oracle's stored res-16 maps
    maps = octrl.attention_store["down_cross"][2:4] + octrl.attention_store["up_cross"][:3]
    maps = np.concatenate([m.reshape(P, -1, 8, 16, 16, 77) for m in maps], axis=2)
    lb = octrl.local_blend
    ref_lb = (maps * lb.alpha_layers).sum(-1).sum(2).reshape(P, F_, 256)
    got_lb = ctrl.attention_store.lb_acc.cpu().numpy()     # (P, f, 256): one word set
    assert np.abs(got_lb - ref_lb).max() / np.abs(ref_lb).max() < tol


def test_unet_forward_inference_mode(tokenizer):
    """a forward under torch.inference_mode() (inference tensors have no version counter,
    so the context / K|V caches must not key on one) runs, twice in a row, and matches the no_grad
    forward.  Not bit for bit: two no_grad forwards of this small config already differ by a bf16 ulp
    here and there (hipBLASLt's stream-K GEMMs on the 256-channel projections accumulate in a
    run-dependent order), so within the bf16 whole-UNet tolerance of test_unet_forward_matches_oracle."""
    unet, sd, ctrl, octrl = _setup(tokenizer, "rabbit", torch.bfloat16)
    x, ctx = _inputs(5)
    x, ctx = x.cuda().bfloat16(), ctx.cuda().bfloat16()
    with torch.no_grad():
        ctrl.cur_step = 0
        ref = unet(x, 981, ctx).sample.float()
    for _ in range(2):
        with torch.inference_mode():
            ctrl.cur_step = 0
            xi, ci = x.clone(), ctx.clone()       # inference tensors
            got = unet(xi, 981, ci).sample
        assert got.is_inference()
        assert _rel(got.float(), ref) < 2e-2, _rel(got.float(), ref)


@pytest.mark.parametrize("substruct", [None, "grass"])
def test_edit_loop_fast_mode(tokenizer, substruct):
    """Three denoising steps through the pipeline (fused CFG + DDIM + LocalBlend) vs the oracle,
    with LocalBlend forced on from the first step (start_blend = 0); optionally with
    LocalBlend(substruct_words=...) (run_videop2p.py:149-151: a second word-weighted sum accumulated
    by K2, thresholded without pooling by K6)."""
    from vp2p.controllers import LocalBlend
    from vp2p.pipeline import VideoP2PPipeline
    unet, sd, ctrl, octrl = _setup(tokenizer, "rabbit", torch.float32, seed=3)
    if substruct:
        prompts = spec.CONFIGS["rabbit"][0]
        sub = ((substruct,), (substruct,))
        ctrl.local_blend = LocalBlend(prompts, (("rabbit",), ("rabbit",)), tokenizer, substruct_words=sub)
        ctrl._plan = None
        octrl.local_blend.substruct_layers = O.LocalBlend._layers(prompts, sub, tokenizer)
        assert ctrl.local_blend.sets == 2
    ctrl.local_blend.start_blend = 0
    octrl.local_blend.start_blend = 0
    x, ctx = _inputs(5)
    x_t = x[:1]
    pipe = VideoP2PPipeline(unet)
    steps = 3
    got = pipe(spec.CONFIGS["rabbit"][0], video_length=F_, height=512, width=512, num_inference_steps=steps,
               latents=x_t.cuda(), controller=ctrl, fast=True, text_embeddings=ctx.cuda()).cpu().numpy()
    d = O.DDIM()
    ts = d.set_timesteps(steps)
    lat = np.repeat(x_t.numpy(), P, axis=0)
    for t in ts:
        eps = unet_ref.unet_forward(sd, torch.from_numpy(np.concatenate([lat, lat])), int(t), ctx, octrl).numpy()
        lat = octrl.step_callback(d.step(O.cfg(eps, 7.5, True), int(t), lat))
    assert np.abs(got - lat).max() / np.abs(lat).max() < 1e-3


@pytest.mark.parametrize("frames", [40, 128])
def test_transformer_long_clip(tokenizer, frames):
    """A Transformer3DModel over a long clip (f > 32: the K3 long-clip kernel behind attn_temp, with
    the self-replace active) vs the oracle transformer (oracle/unet_ref.py, pinned to the reference's
    attention.py) with the oracle controller."""
    import vp2p
    from vp2p.unet3d import Transformer3DModel, init_random_
    prompts, swap, blend, eq, cross, self_ = spec.CONFIGS["rabbit"]
    C, h, w = 320, 4, 4
    m = init_random_(Transformer3DModel(8, C // 8, C, 64), seed=5, std=0.05)
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    m = m.cuda().to(memory_format=torch.channels_last)
    ctrl = vp2p.make_controller(prompts, swap, {"default_": cross}, self_, None, eq, tokenizer=tokenizer)
    octrl = O.EditController(prompts, swap, {"default_": cross}, self_, tokenizer, eq_params=eq)
    holder = torch.nn.Module()
    holder.down_blocks = m                       # registration walks the down*/mid*/up* children
    vp2p.register_attention_control(type("M", (), {"unet": holder})(), ctrl)
    assert ctrl.num_att_layers == 2
    octrl.num_att_layers = 2
    g = np.random.default_rng(9)
    x5 = torch.from_numpy(g.standard_normal((4, C, frames, h, w)).astype(np.float32))
    ctx = torch.from_numpy(g.standard_normal((4, 77, 64)).astype(np.float32))
    ctx[:2] = ctx[0]
    xb = x5.permute(0, 2, 1, 3, 4).reshape(4 * frames, C, h, w).cuda().contiguous(memory_format=torch.channels_last)
    with torch.no_grad():
        got = m(xb, ctx.cuda(), frames).reshape(4, frames, C, h, w).permute(0, 2, 1, 3, 4).cpu()
        ref = unet_ref.transformer(sd, "", x5, ctx, octrl, "down")
    assert ctrl.self_replace_active(frames)
    assert _rel(got, ref) < 2e-4, _rel(got, ref)
