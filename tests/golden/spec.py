"""Shared, seeded definition of the golden-fixture workloads.

``make_golden.py`` (build container only: it executes the reference's own Python from
/root/reference) and the tests both build their inputs from this module, so the committed
``*.npz`` files only need to hold reference OUTPUTS.  All randomness is numpy PCG64
(``np.random.default_rng``), whose streams are stable across processes and machines.

The mini-UNet mirrors the controller-visible structure of the tuneavideo UNet3D: 16 transformer
blocks in down(6) / mid(1) / up(9) order, each with a hooked cross-attention (attn2) followed by a
hooked temporal attention (attn_temp) -> 32 controller calls per forward
(ptp_utils.py:236-255, attention.py:246-268).  Token counts keep the properties the controller
depends on: the "res64" level exceeds the 32**2 store threshold (run_videop2p.py:257), the res16
level has the 16x16 maps LocalBlend reshapes (run_videop2p.py:145-146).
"""
from __future__ import annotations

import numpy as np

HEADS = 8                 # LocalBlend hard-codes 8 heads (run_videop2p.py:146)
DIM_HEAD = 2
C = HEADS * DIM_HEAD      # model channels of the mini blocks
CTX = 24                  # text-embedding width (768 in SD-1.5)
F = 2                     # frames
P = 2                     # prompts (source, edit)
B = 2 * P                 # UNet batch: [uncond x P, cond x P] (pipeline_tuneavideo.py:235)
WORDS = 77
N64, N32, N16, N8 = 1040, 144, 256, 16
LEVELS = [N64, N64, N32, N32, N16, N16, N8, N16, N16, N16, N32, N32, N32, N64, N64, N64]
PLACES = ["down"] * 6 + ["mid"] + ["up"] * 9
NUM_STEPS_SIM = 27        # covers the cross (10) and self (25) window edges
LATENT_HW = 64

SAVE_STEPS = (0, 10, 25)
SAVE_BLOCKS = (4, 6, 7)   # down res16, mid, up res16
LB_SAVE_STEPS = (10, 11, 26)

CONFIGS = {
    # name: (prompts, is_word_swap, blend_words, eq_params, cross_replace_steps, self_replace_steps)
    "rabbit": (["a rabbit is jumping on the grass", "a origami rabbit is jumping on the grass"],
               False, ("rabbit", "rabbit"), {"words": ["origami"], "values": [2]}, 0.2, 0.5),
    "car": (["a car is driving on the road", "a car is driving on the railway"],
            True, ("road", "railway"), {"words": ["railway"], "values": [2]}, 0.2, 0.5),
    "man": (["a man is driving a motorbike in the forest",
             "a Spider-Man is driving a motorbike in the forest"],
            True, ("man", "Spider-Man"), {"words": ["Spider-Man"], "values": [4]}, 0.2, 0.5),
    "penguin": (["a penguin is running on the ice", "a crochet penguin is running on the ice"],
                False, ("penguin", "penguin"), {"words": ["crochet"], "values": [4]}, 0.2, 0.5),
    "bird": (["a bird flying in the forest", "children drawing of a bird flying in the forest"],
             False, None, {"words": ["children", "drawing"], "values": [5, 2]}, 0.8, 0.7),
}
SEQ_CONFIGS = ("rabbit", "car")   # configs driven through the mini-UNet step sequence
BLEND_TOKEN = {"rabbit": (2, 3), "car": (7, 7)}   # token index of blend_word[p] in prompt p
# LocalBlend(substruct_words=...) probe (run_videop2p.py:149-151, 166-174): a word in both prompts
SUBSTRUCT = {"rabbit": "grass", "car": "car"}


def rng(*key: int) -> np.random.Generator:
    return np.random.default_rng(np.random.SeedSequence(list(key)))


def block_weights(cfg_id: int, block: int):
    """Weights of (attn2, attn_temp) of one block: dict of float32 arrays (out, in) like nn.Linear."""
    out = {}
    for li, (name, ctx) in enumerate((("attn2", CTX), ("attn_temp", C))):
        g = rng(11, cfg_id, block, li)
        out[name] = {
            "to_q": (g.standard_normal((C, C)) * 0.25).astype(np.float32),
            "to_k": (g.standard_normal((C, ctx)) * 0.25).astype(np.float32),
            "to_v": (g.standard_normal((C, ctx)) * 0.5).astype(np.float32),
            "to_out_w": (g.standard_normal((C, C)) * 0.4).astype(np.float32),
            "to_out_b": (g.standard_normal((C,)) * 0.1).astype(np.float32),
        }
    return out


def text_embeddings(cfg_id: int) -> np.ndarray:
    """(B, 77, CTX): uncond rows identical (empty prompt), cond rows distinct."""
    g = rng(12, cfg_id)
    unc = g.standard_normal((1, WORDS, CTX)).astype(np.float32)
    cond = g.standard_normal((P, WORDS, CTX)).astype(np.float32)
    for p, tok in enumerate(BLEND_TOKEN[SEQ_CONFIGS[cfg_id]]):
        cond[p, tok] *= 2.5   # the blend word dominates the disk queries (see block_inputs)
    return np.concatenate([np.repeat(unc, P, axis=0), cond], axis=0)


def block_inputs(cfg_id: int, step: int, block: int):
    """Hidden states fed to attn2 ((B*F, N, C), '(b f)' order) and attn_temp ((B*N, F, C), '(b d)')."""
    n = LEVELS[block]
    g = rng(13, cfg_id, step, block)
    x_cross = g.standard_normal((B * F, n, C)).astype(np.float32)
    if n == N16:
        # LocalBlend level: near-uniform attention outside a per-frame disk, a fixed strong query
        # inside it, so the word-weighted maps have spatial structure and the 0.3 threshold
        # (run_videop2p.py:40,138) splits each frame instead of passing everything.
        x1 = rng(16, cfg_id).standard_normal(C).astype(np.float32) * 1.5
        yy, xx = np.mgrid[0:16, 0:16]
        x_cross *= 0.05
        for bf in range(B * F):
            cy = 6.0 + 3.0 * (bf % F)
            disk = ((yy - cy) ** 2 + (xx - cy) ** 2 < 16.0).reshape(-1)
            x_cross[bf, disk] += x1
    x_temp = g.standard_normal((B * n, F, C)).astype(np.float32)
    return x_cross, x_temp


def latents_in(cfg_id: int, step: int) -> np.ndarray:
    """x_t handed to step_callback: (P, 4, F, 64, 64)."""
    g = rng(14, cfg_id, step)
    return g.standard_normal((P, 4, F, LATENT_HW, LATENT_HW)).astype(np.float32)


def controller_probe(kind: str, seed: int):
    """Random softmax maps fed straight to controller(attn, is_cross, place) (cond+uncond batch)."""
    g = rng(15, seed)
    n = 8
    m = WORDS if kind == "cross" else F
    rows = (B * F * HEADS) if kind == "cross" else (B * n * HEADS)
    logits = g.standard_normal((rows, n if kind == "cross" else F, m)).astype(np.float32) * 2.0
    e = np.exp(logits - logits.max(-1, keepdims=True))
    return (e / e.sum(-1, keepdims=True)).astype(np.float32)


PROBE_STEPS = {"cross": (0, 9, 10), "self": (0, 24, 25)}

DDIM_PROBE_T = (981, 501, 21, 1)
