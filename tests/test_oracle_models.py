"""Pin oracle/p2p_oracle.frame_attention and oracle/unet_ref.py to the reference's own model files.

The fixtures (tests/golden/golden_models.npz) are outputs of tuneavideo/models/{attention,resnet,
unet_blocks,unet}.py executed on a restatement of the diffusers-0.11.1 classes they import
(tests/golden/diffusers_shim.py) -- FrameAttention's first-frame K/V gather (attention.py:296-302),
the 5-D GroupNorm of ResnetBlock3D (resnet.py:142,158), the temporal rearrange (attention.py:262-268)
and the block wiring of unet.py:279-414 are the reference's code; the diffusers internals are
restated (parity against the real library unpinned).  CPU only.
"""
import numpy as np
import pytest
import torch

import model_spec as MS
from conftest import model_state
from oracle import p2p_oracle as O
from oracle import unet_ref



@pytest.fixture(autouse=True)
def _no_grad():
    """Grad off inside this module's tests only (a module-level set_grad_enabled(False) would leak
    into every test collected after it, e.g. the GPU backward tests of the same session)."""
    with torch.no_grad():
        yield


@pytest.mark.parametrize("name", list(MS.FA_CONFIGS))
def test_frame_attention_pinned(golden_models, name):
    """p2p_oracle.frame_attention + the projections == the reference FrameAttention (attention.py:273-329)."""
    B, f, N, C = MS.FA_CONFIGS[name]
    w = {k: MS.param_values(k, s, 41).astype(np.float64) for k, s in
         (("to_q.weight", (C, C)), ("to_k.weight", (C, C)), ("to_v.weight", (C, C)),
          ("to_out.0.weight", (C, C)), ("to_out.0.bias", (C,)))}
    x = MS.fa_input(name)
    q, k, v = (x @ w[f"to_{n}.weight"].T for n in "qkv")
    core = O.frame_attention(q.astype(np.float32), k.astype(np.float32), v.astype(np.float32), f, MS.HEADS)
    out = core @ w["to_out.0.weight"].T + w["to_out.0.bias"]
    np.testing.assert_allclose(out, golden_models[f"fa/{name}"], rtol=1e-4, atol=2e-5)


def _t3d_factory(C, D):
    from vp2p.unet3d import Transformer3DModel
    return lambda: Transformer3DModel(MS.HEADS, C // MS.HEADS, C, D)


@pytest.mark.parametrize("name", list(MS.T3D_CONFIGS))
def test_transformer3d_pinned(golden_models, name):
    """unet_ref.transformer (hooked attn2/attn_temp under the DummyController) == the reference
    Transformer3DModel with ptp_utils.register_attention_control(model, None) applied, and == the
    un-hooked diffusers attention (the two softmaxes agree in the finite regime)."""
    B, f, h, w, C, D = MS.T3D_CONFIGS[name]
    sd = model_state(_t3d_factory(C, D), 42)
    x, ctx = (torch.from_numpy(a) for a in MS.t3d_inputs(name))
    got = unet_ref.transformer(sd, "", x, ctx, None, "down").numpy()
    np.testing.assert_allclose(got, golden_models[f"t3d/{name}/hooked"], rtol=1e-4, atol=5e-5)
    np.testing.assert_allclose(got, golden_models[f"t3d/{name}/plain"], rtol=1e-4, atol=5e-5)


@pytest.mark.parametrize("name", list(MS.RN_CONFIGS))
def test_resnet3d_pinned(golden_models, name):
    """unet_ref.resnet == the reference ResnetBlock3D (5-D GroupNorm over c/G x f x h x w)."""
    from vp2p.unet3d import ResnetBlock3D
    B, f, h, w, cin, cout, T = MS.RN_CONFIGS[name]
    sd = model_state(lambda: ResnetBlock3D(cin, cout, T), 43)
    x, temb = (torch.from_numpy(a) for a in MS.rn_inputs(name))
    got = unet_ref.resnet(sd, "", x, temb).numpy()
    np.testing.assert_allclose(got, golden_models[f"rn/{name}"], rtol=1e-4, atol=5e-5)


@pytest.fixture(scope="module")
def sd_unet():
    from vp2p.unet3d import UNet3DConditionModel
    return model_state(UNet3DConditionModel, 44)


def test_unet_sd15_geometry_pinned(golden_models, sd_unet):
    """unet_ref.unet_forward at the SD-1.5 channel layout (320/640/1280/1280, d = 40/80/160) ==
    the reference UNet3DConditionModel under the DummyController hook (inversion's registration,
    run_videop2p.py:628)."""
    sample, ctx = (torch.from_numpy(a) for a in MS.unet_small_inputs())
    got = unet_ref.unet_forward(sd_unet, sample, MS.UNET_SMALL_T, ctx).numpy()
    np.testing.assert_allclose(got, golden_models["unet/dummy"], rtol=1e-4, atol=5e-5)


@pytest.mark.parametrize("step", MS.UNET_EDIT_STEPS)
def test_unet_controlled_pinned(golden_models, sd_unet, tokenizer, step):
    """unet_ref with the oracle controller == the reference UNet with the reference controller
    (bird: AttentionRefine + Reweight, cross 0.8, self 0.7) at controller step ``step``."""
    import spec
    prompts, swap, blend, eq, cross, self_ = spec.CONFIGS["bird"]
    ctrl = O.EditController(prompts, swap, {"default_": cross}, self_, tokenizer, blend_words=None, eq_params=eq)
    ctrl.cur_step = step
    sample, ctx = (torch.from_numpy(a) for a in MS.unet_small_inputs(4))
    got = unet_ref.unet_forward(sd_unet, sample, MS.UNET_SMALL_T, ctx, controller=ctrl).numpy()
    assert int(golden_models[f"unet/bird/{step}/layers"]) == 32
    np.testing.assert_allclose(got, golden_models[f"unet/bird/{step}"], rtol=1e-4, atol=5e-5)


@pytest.fixture(scope="module")
def golden_nulltext():
    import os
    from conftest import ROOT
    return np.load(os.path.join(ROOT, "tests", "golden", "golden_nulltext.npz"))


def test_null_optimization_pinned(golden_nulltext):
    """unet_ref.null_optimization (the CPU restatement of run_videop2p.py:580-612) == the reference's
    own NullInversion.ddim_loop + null_optimization (AST-extracted, run on the reference UNet;
    tests/golden/make_golden_models.py --part nulltext) on the 256/512-channel config: every inner
    loss, the optimised unconditional embeddings and the inversion latents."""
    from vp2p.unet3d import UNet3DConditionModel, init_random_
    cfg, std, _, steps, inner = MS.NULLTEXT["c256"]
    sd = init_random_(UNet3DConditionModel(**cfg), seed=0, std=std).state_dict()
    x0, ctx = (torch.from_numpy(a) for a in MS.nulltext_inputs("c256"))
    ddim = O.DDIM()
    ddim.set_timesteps(steps)
    lats = [x0]
    ts = [int(t) for t in ddim.timesteps]
    for i in range(steps):       # NullInversion.ddim_loop (run_videop2p.py:557-567)
        t = ts[len(ts) - i - 1]
        lats.append(ddim.next_step(unet_ref.unet_forward(sd, lats[-1], t, ctx[1:]).numpy(), t,
                                   lats[-1].numpy()))
        lats[-1] = torch.from_numpy(np.asarray(lats[-1], np.float32))
    ref_lats = golden_nulltext["c256/latents"]
    np.testing.assert_allclose(torch.stack(lats).numpy(), ref_lats, rtol=1e-4, atol=1e-5)
    with torch.enable_grad():
        unc, losses, _ = unet_ref.null_optimization(sd, [torch.from_numpy(a) for a in ref_lats], ctx[:1], ctx[1:],
                                                    ddim, num_inner_steps=inner)
    np.testing.assert_allclose(losses, golden_nulltext["c256/losses"], rtol=1e-4)
    # Adam divides by sqrt(v): an element whose gradient is ~0 moves by up to lr per iteration with a
    # sign set by rounding noise, so a few elements may differ by a fraction of lr (1e-2)
    diff = np.abs(torch.cat(unc).numpy() - golden_nulltext["c256/uncond"])
    assert diff.mean() < 1e-5 and diff.max() < 1e-2, (diff.mean(), diff.max())


@pytest.mark.parametrize("name", list(MS.T3D_CONFIGS))
def test_transformer_token_slice_pinned(golden_models, name):
    """unet_ref.transformer_token_slice (the long-clip oracle: Transformer3DModel at a few positions of
    every frame) == the reference Transformer3DModel (attention.py:90-137) at those positions."""
    B, f, h, w, C, D = MS.T3D_CONFIGS[name]
    sd = model_state(_t3d_factory(C, D), 42)
    x, ctx = (torch.from_numpy(a) for a in MS.t3d_inputs(name))
    tokens = [0, 3, h * w // 2 + 1, h * w - 1]
    got = unet_ref.transformer_token_slice(sd, "", x, ctx, tokens).numpy()
    ref = golden_models[f"t3d/{name}/hooked"].reshape(B, C, f, h * w)[..., tokens]
    np.testing.assert_allclose(got, ref, rtol=1e-4, atol=5e-5)
