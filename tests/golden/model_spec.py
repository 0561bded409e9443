"""Seeded definition of the MODEL-level golden fixtures (``golden_models.npz``, ``golden_edit_*.npz``).

``make_golden_models.py`` (build container only) runs the reference's own tuneavideo model files
and TuneAVideoPipeline loop on these inputs; the tests regenerate the same inputs and weights from
this module, so the committed fixtures hold only reference OUTPUTS.

Weights: ``fill_`` draws every state-dict entry from its own numpy PCG64 stream keyed by
(seed, crc32(name)), so the values depend only on the parameter's name and shape -- the
reference's modules and vp2p's (same state-dict keys) receive identical weights whatever order
their constructors register them in.  The SD-1.5-geometry edit fixtures use
``vp2p.unet3d.init_random_`` instead (the bench's weights; torch's CPU generator, identical on
this image and the GPU box).
"""
from __future__ import annotations

import zlib
from typing import Dict

import numpy as np

HEADS = 8

# FrameAttention (attention.py:273-329): name -> (batch, frames, tokens, channels); head dim = C/8
FA_CONFIGS = {"d40": (2, 3, 80, 320), "d80": (1, 4, 64, 640), "d160": (2, 2, 48, 1280)}
# Transformer3DModel (attention.py:32-137): name -> (batch, frames, h, w, channels, cross_dim)
T3D_CONFIGS = {"c320": (2, 3, 8, 8, 320, 768), "c640": (2, 2, 4, 6, 640, 768)}
# ResnetBlock3D (resnet.py:111-205): name -> (batch, frames, h, w, cin, cout, temb)
RN_CONFIGS = {"c320_640": (2, 3, 8, 8, 320, 640, 1280), "c640": (2, 2, 4, 4, 640, 640, 1280)}
# Whole UNet3DConditionModel at the SD-1.5 geometry (unet.py:42-79 defaults, cross dim 768) on a
# small latent: (batch, frames, latent h, latent w)
UNET_SMALL = (2, 2, 16, 16)
UNET_SMALL_T = 501
UNET_EDIT_STEPS = (0, 45)          # controller cur_step of the two controlled forwards (bird edit)

# End-to-end edits through the reference pipeline loop (pipeline_tuneavideo.py:394-430):
# name -> (edit, frames, steps run of the 50-step schedule, steps whose latents are saved)
EDITS = {
    "car2": ("car", 2, 12, (0, 9, 10, 11)),
    "rabbit8": ("rabbit", 8, 50, (0, 10, 11, 24, 25, 49)),
    # configs[2], all 50 steps: across the self-replace boundary (self_replace_steps 0.5 of 50: steps
    # 24 / 25) and through the last LocalBlend-driven step 49 (round 6; round 5's fixture stopped at
    # step 26, round 3's "penguin24" at step 11)
    "penguin24l": ("penguin", 24, 50, (10, 11, 24, 25, 26, 49)),
}


def edit_schedule(name: str, gold=None):
    """(steps to run, steps whose latents are compared) for an end-to-end edit: from the fixture when
    one is given (its ``steps_run`` and saved ``latents/<i>``), so a fixture generated for an older
    EDITS entry still checks what it holds; else EDITS[name]."""
    _, _, steps, save = EDITS[name]
    if gold is not None:
        steps = int(gold["steps_run"])
        save = tuple(sorted(int(k.split("/")[1]) for k in gold.files if k.startswith("latents/")))
    return steps, save


# Null-text optimisation fixtures (run_videop2p.py:557-612): name -> (UNet3DConditionModel kwargs,
# init_random_ std, x_0 shape (1, 4, f, h, w), DDIM steps, max inner Adam iterations)
NULLTEXT = {
    "c256": (dict(block_out_channels=(256, 256, 512, 512), cross_attention_dim=64, attention_head_dim=8),
             0.05, (1, 4, 2, 32, 32), 2, 3),
    "sd15": (dict(cross_attention_dim=768), 0.02, (1, 4, 2, 16, 16), 2, 3),
    # configs[3]'s frame count at SD-1.5 geometry (8 frames; 32^2 latents keep the CPU reference run
    # to minutes): the sharded-frame and real-size backward pin (VERDICT r03 "backward at real size")
    "sd15f8": (dict(cross_attention_dim=768), 0.02, (1, 4, 8, 32, 32), 2, 3),
}


def rng(*key: int) -> np.random.Generator:
    return np.random.default_rng(np.random.SeedSequence(list(key)))


def param_values(name: str, shape, seed: int) -> np.ndarray:
    """Deterministic value of one state-dict entry.  Weights ~ N(0, 1/fan_in) (unit-gain
    projections, so activations neither vanish nor blow up through the blocks), biases ~ N(0, 0.1^2),
    norm scales ~ 1 + N(0, 0.1^2), norm shifts ~ N(0, 0.1^2)."""
    g = rng(seed, zlib.crc32(name.encode()))
    shape = tuple(shape)
    leaf = name.rsplit(".", 1)[-1]
    is_norm = "norm" in name.rsplit(".", 2)[-2] if name.count(".") >= 1 else False
    if leaf == "weight" and is_norm:
        v = 1.0 + 0.1 * g.standard_normal(shape)
    elif leaf == "bias":
        v = 0.1 * g.standard_normal(shape)
    else:
        fan_in = int(np.prod(shape[1:])) if len(shape) > 1 else 1
        v = g.standard_normal(shape) / np.sqrt(fan_in)
    return v.astype(np.float32)


def fill_(module, seed: int):
    """Overwrite every parameter of ``module`` (a torch nn.Module) with ``param_values``."""
    import torch
    with torch.no_grad():
        for name, p in module.state_dict().items():
            if p.dtype.is_floating_point:
                p.copy_(torch.from_numpy(param_values(name, p.shape, seed)))
    return module


def fa_input(name: str) -> np.ndarray:
    B, f, N, C = FA_CONFIGS[name]
    return rng(31, zlib.crc32(name.encode())).standard_normal((B * f, N, C)).astype(np.float32)


def t3d_inputs(name: str):
    """(hidden (B, C, f, h, w), context (B, 77, D))."""
    B, f, h, w, C, D = T3D_CONFIGS[name]
    g = rng(32, zlib.crc32(name.encode()))
    return (g.standard_normal((B, C, f, h, w)).astype(np.float32),
            g.standard_normal((B, 77, D)).astype(np.float32))


def rn_inputs(name: str):
    """(hidden (B, Cin, f, h, w), temb (B, T))."""
    B, f, h, w, cin, cout, T = RN_CONFIGS[name]
    g = rng(33, zlib.crc32(name.encode()))
    return g.standard_normal((B, cin, f, h, w)).astype(np.float32), g.standard_normal((B, T)).astype(np.float32)


def nulltext_inputs(name: str):
    """(x_0 (1, 4, f, h, w), context [uncond; cond] (2, 77, D)) of one null-text fixture."""
    cfg, _, shape, _, _ = NULLTEXT[name]
    g = rng(36, zlib.crc32(name.encode()))
    return (g.standard_normal(shape).astype(np.float32),
            g.standard_normal((2, 77, cfg["cross_attention_dim"])).astype(np.float32))


def unet_small_inputs(batch: int = None):
    """(sample (B, 4, f, h, w), context (B, 77, 768)); ``batch`` overrides B (4 for the edit forwards:
    rows [uncond x 2, cond x 2] with identical uncond rows)."""
    B, f, h, w = UNET_SMALL
    B = batch or B
    g = rng(34, B)
    sample = g.standard_normal((B, 4, f, h, w)).astype(np.float32)
    ctx = g.standard_normal((B, 77, 768)).astype(np.float32)
    if B == 4:
        sample[1] = sample[0]
        sample[3] = sample[2]
        ctx[1] = ctx[0]
    return sample, ctx


# The end-to-end edits must exercise LocalBlend with NON-trivial masks (run_videop2p.py:131-154: the
# blend is the identity when every pixel passes `mask / max > th`).  With i.i.d. N(0, 0.02) weights
# and white-noise latents the 40 res-16 cross maps LocalBlend averages are independent and spatially
# white, so after the 3x3 max-pool every pixel passes.  Three changes make the maps agree and
# localise, as a trained model's do (profiles/r03_mask_localisation.txt):
#   * x_T is spatially smooth (an EDIT_LOWRES^2 N(0, 1) grid per channel and frame, bicubic-upsampled
#     to 64^2, unit std) instead of white noise;
#   * the 5 res-16 attn2 layers LocalBlend reads share one (head-0, first-layer) to_q / to_k block
#     across their 8 heads (``edit_state``), so the 40 maps are 5 maps of one query/key geometry;
#   * the blend words' conditional text embeddings are scaled by EDIT_BLEND_SCALE.
EDIT_LOWRES = 6
EDIT_BLEND_SCALE = 4.0
RES16_ATTN2 = ["down_blocks.2.attentions.0", "down_blocks.2.attentions.1", "up_blocks.1.attentions.0",
               "up_blocks.1.attentions.1", "up_blocks.1.attentions.2"]


def edit_state(sd):
    """The edit fixtures' UNet weights: the bench's (``vp2p.unet3d.init_random_`` seed 0) with the
    res-16 attn2 to_q / to_k tied as described above.  ``sd``: {name: CPU tensor}; returns a new dict."""
    out = dict(sd)
    for nm in ("to_q", "to_k"):
        src = sd[f"{RES16_ATTN2[0]}.transformer_blocks.0.attn2.{nm}.weight"]
        d = src.shape[0] // HEADS
        tied = src[:d].repeat(HEADS, 1).contiguous()
        for layer in RES16_ATTN2:
            out[f"{layer}.transformer_blocks.0.attn2.{nm}.weight"] = tied.clone()
    return out


def edit_inputs(name: str, blend_token_ids=None) -> Dict[str, np.ndarray]:
    """x_T (1, 4, f, 64, 64) and the CFG text embeddings [uncond, uncond, cond_0, cond_1] (4, 77, 768)
    of one end-to-end edit.  ``blend_token_ids``: per prompt, the token indices of its blend word
    (``get_word_inds``), whose conditional embeddings are scaled by EDIT_BLEND_SCALE."""
    import torch
    _, f, _, _ = EDITS[name]
    g = rng(35, zlib.crc32(name.encode()))
    lo = torch.from_numpy(g.standard_normal((1, 4 * f, EDIT_LOWRES, EDIT_LOWRES)).astype(np.float32))
    x = torch.nn.functional.interpolate(lo, size=(64, 64), mode="bicubic", align_corners=False)
    x_t = (x / x.std()).reshape(1, 4, f, 64, 64).numpy().astype(np.float32)
    unc = g.standard_normal((1, 77, 768)).astype(np.float32)
    cond = g.standard_normal((2, 77, 768)).astype(np.float32)
    if blend_token_ids is not None:
        for p, ids in enumerate(blend_token_ids):
            cond[p, list(ids)] *= np.float32(EDIT_BLEND_SCALE)
    return {"x_t": x_t, "emb": np.concatenate([unc, unc, cond]).astype(np.float32)}


def blend_token_ids(prompts, blend, tokenizer):
    """Token indices of each prompt's blend word (vp2p.prompt_align.get_word_inds, golden-exact
    against ptp_utils.get_word_inds)."""
    from vp2p.prompt_align import get_word_inds
    return [tuple(int(i) for i in get_word_inds(p, w, tokenizer)) for p, w in zip(prompts, blend)]
