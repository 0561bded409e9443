"""GPU parity against the REFERENCE's own model files and pipeline loop (no oracle in between).

Fixtures: tests/golden/golden_models.npz and golden_edit_*.npz, written by
tests/golden/make_golden_models.py from tuneavideo/models/*.py, ptp_utils.py, run_videop2p.py's
controllers and TuneAVideoPipeline.__call__ (pipeline_tuneavideo.py:394-430), all fp32 on the CPU.

Tolerances (BASELINE.json north_star): attention-level outputs within 1e-4 relative in fp32 and
2e-2 in bf16.  Multi-layer outputs (a transformer block, a resnet, the whole UNet, an edit) are
reported as max-abs error relative to the reference's max |value| ("rel") and as PSNR
= 10 log10(max(ref^2) / mean((got - ref)^2)); the bars are stated per test below and in DESIGN.md §2.
"""
import os

import numpy as np
import pytest
import torch

import model_spec as MS
from conftest import ROOT, model_state, record

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(ROOT, "tests", "golden")


def _rel(a, b):
    return float(np.abs(a - b).max() / np.abs(b).max())


def psnr(got, ref):
    got, ref = np.asarray(got, np.float64), np.asarray(ref, np.float64)
    return float(10 * np.log10((ref ** 2).max() / max(((got - ref) ** 2).mean(), 1e-30)))


def _load_module(module, sd, dtype):
    module.load_state_dict(sd, strict=True)
    return module.to("cuda", dtype).to(memory_format=torch.channels_last).eval()


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-4), (torch.bfloat16, 2e-2)])
@pytest.mark.parametrize("name", list(MS.FA_CONFIGS))
def test_frame_attention_vs_reference(golden_models, name, dtype, tol):
    """vp2p FrameAttention (K1, projections on hipBLASLt) vs the reference FrameAttention
    (attention.py:273-329) at head dims 40 / 80 / 160 (the SD-1.5 levels)."""
    from vp2p.attention import FrameAttention
    B, f, N, C = MS.FA_CONFIGS[name]
    fa = lambda: FrameAttention(C, heads=MS.HEADS, dim_head=C // MS.HEADS)  # noqa: E731
    m = _load_module(fa(), model_state(fa, 41), dtype)
    x = torch.from_numpy(MS.fa_input(name)).cuda().to(dtype)
    with torch.no_grad():
        got = m(x, video_length=f).float().cpu().numpy()
    record(f"frame_attention/{name}/{dtype}", rel=_rel(got, golden_models[f"fa/{name}"]), tol=tol)
    assert _rel(got, golden_models[f"fa/{name}"]) < tol, _rel(got, golden_models[f"fa/{name}"])


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-4), (torch.bfloat16, 2e-2)])
@pytest.mark.parametrize("name", list(MS.T3D_CONFIGS))
def test_transformer3d_vs_reference(golden_models, name, dtype, tol):
    """One full Transformer3DModel (GroupNorm, proj_in, attn1/K1, attn2/K2, GEGLU FF, attn_temp/K3,
    proj_out + residual) at the real SD-1.5 channel counts and head dims."""
    from vp2p.unet3d import Transformer3DModel
    B, f, h, w, C, D = MS.T3D_CONFIGS[name]
    fac = lambda: Transformer3DModel(MS.HEADS, C // MS.HEADS, C, D)  # noqa: E731
    m = _load_module(fac(), model_state(fac, 42), dtype)
    x, ctx = MS.t3d_inputs(name)
    xb = torch.from_numpy(x).permute(0, 2, 1, 3, 4).reshape(B * f, C, h, w)
    xb = xb.cuda().to(dtype).contiguous(memory_format=torch.channels_last)
    with torch.no_grad():
        y = m(xb, torch.from_numpy(ctx).cuda().to(dtype), f)
    got = y.float().reshape(B, f, C, h, w).permute(0, 2, 1, 3, 4).cpu().numpy()
    ref = golden_models[f"t3d/{name}/hooked"]
    record(f"transformer3d/{name}/{dtype}", rel=_rel(got, ref), psnr=psnr(got, ref), tol=tol)
    assert _rel(got, ref) < tol, _rel(got, ref)


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-4), (torch.bfloat16, 2e-2)])
@pytest.mark.parametrize("name", list(MS.RN_CONFIGS))
def test_resnet3d_vs_reference(golden_models, name, dtype, tol):
    """ResnetBlock3D (K7 5-D GroupNorm + SiLU + temb add, K10 / MIOpen convs, fused shortcut add)."""
    from vp2p.unet3d import ResnetBlock3D
    B, f, h, w, cin, cout, T = MS.RN_CONFIGS[name]
    fac = lambda: ResnetBlock3D(cin, cout, T)  # noqa: E731
    m = _load_module(fac(), model_state(fac, 43), dtype)
    x, temb = MS.rn_inputs(name)
    xb = torch.from_numpy(x).permute(0, 2, 1, 3, 4).reshape(B * f, cin, h, w)
    xb = xb.cuda().to(dtype).contiguous(memory_format=torch.channels_last)
    with torch.no_grad():
        y = m(xb, torch.from_numpy(temb).cuda().to(dtype), f)
    got = y.float().reshape(B, f, cout, h, w).permute(0, 2, 1, 3, 4).cpu().numpy()
    record(f"resnet3d/{name}/{dtype}", rel=_rel(got, golden_models[f"rn/{name}"]),
           psnr=psnr(got, golden_models[f"rn/{name}"]), tol=tol)
    assert _rel(got, golden_models[f"rn/{name}"]) < tol, _rel(got, golden_models[f"rn/{name}"])


@pytest.fixture(scope="module")
def sd15_state():
    from vp2p.unet3d import UNet3DConditionModel
    return model_state(UNet3DConditionModel, 44)


# whole UNet (60+ layers): fp32 within 1e-4 of the reference's max; bf16 PSNR >= 44 dB (measured 47-48)
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_unet_sd15_vs_reference(golden_models, sd15_state, dtype):
    """The SD-1.5-geometry UNet3D (d = 40 / 80 / 160, 16 transformer blocks, 22 resnets) on a
    16x16 latent vs the reference UNet3DConditionModel under the DummyController hook."""
    from vp2p.unet3d import UNet3DConditionModel
    m = _load_module(UNet3DConditionModel(), sd15_state, dtype)
    sample, ctx = MS.unet_small_inputs()
    with torch.no_grad():
        got = m(torch.from_numpy(sample).cuda().to(dtype), MS.UNET_SMALL_T,
                torch.from_numpy(ctx).cuda().to(dtype)).sample.float().cpu().numpy()
    ref = golden_models["unet/dummy"]
    record(f"unet_sd15/{dtype}", rel=_rel(got, ref), psnr=psnr(got, ref))
    if dtype == torch.float32:
        assert _rel(got, ref) < 1e-4, _rel(got, ref)
    else:
        assert psnr(got, ref) >= 44.0, psnr(got, ref)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("step", MS.UNET_EDIT_STEPS)
def test_unet_controlled_vs_reference(golden_models, sd15_state, tokenizer, dtype, step):
    """The same UNet under the fused P2P controller (bird: AttentionRefine + AttentionReweight on two
    words, cross 0.8 / self 0.7) vs the reference controller registered by ptp_utils at step ``step``."""
    import spec
    import vp2p
    from vp2p.unet3d import UNet3DConditionModel
    m = _load_module(UNet3DConditionModel(), sd15_state, dtype)
    prompts, swap, blend, eq, cross, self_ = spec.CONFIGS["bird"]
    ctrl = vp2p.make_controller(prompts, swap, {"default_": cross}, self_, None, eq, tokenizer=tokenizer)
    vp2p.register_attention_control(type("M", (), {"unet": m})(), ctrl)
    assert ctrl.num_att_layers == int(golden_models[f"unet/bird/{step}/layers"])
    ctrl.cur_step = step
    sample, ctx = MS.unet_small_inputs(4)
    with torch.no_grad():
        got = m(torch.from_numpy(sample).cuda().to(dtype), MS.UNET_SMALL_T,
                torch.from_numpy(ctx).cuda().to(dtype)).sample.float().cpu().numpy()
    ref = golden_models[f"unet/bird/{step}"]
    assert ctrl.cur_step == step + 1 and ctrl.cur_att_layer == 0
    record(f"unet_sd15_bird/{step}/{dtype}", rel=_rel(got, ref), psnr=psnr(got, ref))
    if dtype == torch.float32:
        assert _rel(got, ref) < 1e-4, _rel(got, ref)
    else:
        assert psnr(got, ref) >= 44.0, psnr(got, ref)


# -- end-to-end edits ---------------------------------------------------------------------------------
@pytest.fixture(scope="module")
def bench_state():
    """The bench's SD-1.5 weights (init_random_ seed 0), built once on the CPU."""
    from vp2p.unet3d import UNet3DConditionModel, init_random_
    return init_random_(UNet3DConditionModel(), seed=0).state_dict()


def run_edit(name, dtype, tokenizer, state, schedule=None):
    """vp2p's fast-mode edit of model_spec.EDITS[name] (the fixture's weights and inputs:
    model_spec.edit_state / edit_inputs); returns ({step: latents}, {step: the LocalBlend mask K6
    applied that step}, controller).  The mask is K6's own output (``VideoP2PPipeline.keep_blend_mask``
    -> vp2p_step_args.mask_out), not a host recomputation from the LocalBlend sums."""
    import spec
    import vp2p
    from vp2p.pipeline import VideoP2PPipeline
    from vp2p.unet3d import UNet3DConditionModel
    edit, f, _, _ = MS.EDITS[name]
    steps, save = schedule if schedule is not None else MS.edit_schedule(name)
    prompts, swap, blend, eq, cross, self_ = spec.CONFIGS[edit]
    unet = UNet3DConditionModel()
    unet.load_state_dict(MS.edit_state(state), strict=True)
    unet = unet.to("cuda", dtype).to(memory_format=torch.channels_last).eval()
    ctrl = vp2p.make_controller(prompts, swap, {"default_": cross}, self_, ((blend[0],), (blend[1],)), eq,
                                tokenizer=tokenizer)
    vp2p.register_attention_control(type("M", (), {"unet": unet})(), ctrl)
    inp = MS.edit_inputs(name, MS.blend_token_ids(prompts, blend, tokenizer))
    lats, masks = {}, {}
    pipe = VideoP2PPipeline(unet)
    pipe.keep_blend_mask = True

    class Stop(Exception):
        pass

    def cb(i, t, lat):
        if i in save:
            lats[i] = lat.cpu().numpy()
            if ctrl.local_blend.counter > ctrl.local_blend.start_blend:
                masks[i] = pipe.blend_mask.cpu().numpy().astype(bool)
        if i == steps - 1:
            raise Stop

    try:
        with torch.no_grad():
            pipe(prompts, f, latents=torch.from_numpy(inp["x_t"]).cuda(), controller=ctrl, fast=True,
                 text_embeddings=torch.from_numpy(inp["emb"]).cuda(), num_inference_steps=50, callback=cb)
    except Stop:
        pass
    return lats, masks, ctrl


def _edit_fixture(name):
    path = os.path.join(GOLDEN, f"golden_edit_{name}.npz")
    if not os.path.exists(path):
        pytest.skip(f"{path} not generated (tests/golden/make_golden_models.py --part {name})")
    return np.load(path)


# End-to-end bars: fp32 -- final-latent PSNR >= 100 dB and K6's applied LocalBlend masks
# equal to the reference's (0 flips); bf16 -- final-latent PSNR >= 45 dB and at
# most 2% of the mask pixels flipped.  Every saved reference mask is non-trivial (true fraction in
# [0.05, 0.95], asserted by the generator and here; the blend maps are summed over steps, so late masks
# that widen past 0.95 are not saved, only their fraction -- the first blend step's mask always is).
# The fp32 rabbit8 case runs 50 fp32 UNet steps (~145 s, profiles/r02_edit_pipeline_durations.log),
# more than a 120 s per-test limit on the command line allows.
# penguin24l (configs[2], 24 frames): all 50 steps, latents saved at 10 / 11 (the first blend steps),
# 24 / 25 / 26 (across the self-replace boundary) and 49 (the final latents); the schedule comes from
# the fixture itself (model_spec.edit_schedule).  In fp32 (the reference's precision) its
# convolutions run on MIOpen (K10 is bf16), whose compiled kernels for the 24-frame shapes come from the
# in-tree cache (miopen_db/kcache, vp2p.tuning) instead of minutes of compiling on a fresh box.
EDIT_CASES = [pytest.param(n, dt, bar, id=f"{n}-{'fp32' if dt == torch.float32 else 'bf16'}")
              for n, dt, bar in (("car2", torch.float32, 100.0), ("car2", torch.bfloat16, 45.0),
                                 ("rabbit8", torch.float32, 100.0), ("rabbit8", torch.bfloat16, 45.0),
                                 ("penguin24l", torch.float32, 100.0), ("penguin24l", torch.bfloat16, 45.0))]


@pytest.mark.timeout(600)
@pytest.mark.parametrize("name,dtype,bar", EDIT_CASES)
def test_edit_vs_reference_pipeline(tokenizer, bench_state, name, dtype, bar):
    gold = _edit_fixture(name)
    steps, save = MS.edit_schedule(name, gold)
    lats, masks, ctrl = run_edit(name, dtype, tokenizer, bench_state, (steps, save))
    assert ctrl.cur_step == int(gold["cur_step"]) and ctrl.local_blend.counter == int(gold["lb_counter"])
    report = []
    n_masks = 0
    for i in save:
        p = psnr(lats[i], gold[f"latents/{i}"])
        report.append((i, round(p, 1)))
        if f"mask/{i}" in gold.files:
            n_masks += 1
            ref_mask = np.unpackbits(gold[f"mask/{i}"])[: masks[i].size].reshape(masks[i].shape).astype(bool)
            frac = ref_mask.reshape(ref_mask.shape[0], -1).mean(1)
            assert ((frac >= 0.05) & (frac <= 0.95)).all(), f"vacuous reference mask at step {i}: {frac}"
            flips = int((masks[i] != ref_mask).sum())
            report.append((i, "mask flips", flips, masks[i].size, "ref true frac", [round(float(x), 3) for x in frac]))
            # fp32: bit-exact (0 flips: the north star's "LocalBlend masks bit-exact after thresholding at
            # fp32"; measured 0 on every fixture since round 2); bf16: at most 2% (measured 0.1-0.9%,
            # profiles/r04_parity.jsonl)
            assert flips <= (0 if dtype == torch.float32 else masks[i].size // 50), report
    assert n_masks > 0, "fixture holds no LocalBlend mask"
    record(f"edit/{name}/{dtype}", steps=report, final_psnr=psnr(lats[save[-1]], gold[f"latents/{save[-1]}"]),
           bar=bar)
    assert psnr(lats[save[-1]], gold[f"latents/{save[-1]}"]) >= bar, report
