"""Pin the CPU oracle to the reference's own outputs (tests/golden/golden.npz)."""
import numpy as np
import pytest

import spec
from oracle import p2p_oracle as O


def _cfg(name):
    prompts, swap, blend, eq, cross, self_ = spec.CONFIGS[name]
    return prompts, swap, blend, eq, cross, self_


@pytest.mark.parametrize("name", list(spec.CONFIGS))
def test_host_logic(golden, tokenizer, name):
    prompts, swap, blend, eq, cross, self_ = _cfg(name)
    m, a = O.refinement_mapper(prompts, tokenizer)
    np.testing.assert_array_equal(m, golden[f"{name}/refine_mapper"])
    np.testing.assert_array_equal(a, golden[f"{name}/refine_alphas"])
    if swap:
        np.testing.assert_array_equal(O.replacement_mapper(prompts, tokenizer),
                                      golden[f"{name}/replace_mapper"])
    np.testing.assert_array_equal(O.time_word_alpha(prompts, 50, {"default_": cross}, tokenizer),
                                  golden[f"{name}/cross_replace_alpha"])
    np.testing.assert_array_equal(O.equalizer(prompts[1], eq["words"], eq["values"], tokenizer),
                                  golden[f"{name}/equalizer"])
    if blend is not None:
        for i, w in enumerate(blend):
            np.testing.assert_array_equal(O.get_word_inds(prompts[i], w, tokenizer),
                                          golden[f"{name}/word_inds_{i}"])


def test_alpha_word_override_and_errors(golden, tokenizer):
    prompts = spec.CONFIGS["rabbit"][0]
    got = O.time_word_alpha(prompts, 50, {"default_": 0.2, "origami": (0.1, 0.6)}, tokenizer)
    np.testing.assert_array_equal(got, golden["misc/alpha_word_override"])
    assert int(golden["misc/replace_unequal_raises"]) == 1
    with pytest.raises(ValueError):
        O.replacement_mapper(prompts, tokenizer)


@pytest.mark.parametrize("name", list(spec.SEQ_CONFIGS) + ["man", "penguin", "bird"])
@pytest.mark.parametrize("kind", ["cross", "self"])
def test_controller_probes(golden, tokenizer, name, kind):
    prompts, swap, blend, eq, cross, self_ = _cfg(name)
    ci = (list(spec.SEQ_CONFIGS) + ["man", "penguin", "bird"]).index(name)
    for s in spec.PROBE_STEPS[kind]:
        ctrl = O.EditController(prompts, swap, {"default_": cross}, self_, tokenizer,
                                blend_words=None if blend is None else ((blend[0],), (blend[1],)),
                                eq_params=eq)
        ctrl.cur_step = s
        attn = spec.controller_probe(kind, 100 * ci + s)
        got = ctrl(attn, kind == "cross", "up")
        np.testing.assert_allclose(got, golden[f"probe/{name}/{kind}/{s}"], rtol=1e-6, atol=1e-7)


def _mini_unet_weights(cfg_id):
    return [spec.block_weights(cfg_id, b) for b in range(16)]


@pytest.mark.parametrize("cfg_id,name", list(enumerate(spec.SEQ_CONFIGS)))
def test_step_sequence(golden, tokenizer, cfg_id, name):
    """Hooked forward + controller + LocalBlend over 27 steps of the 32-layer call sequence."""
    prompts, swap, blend, eq, cross, self_ = _cfg(name)
    ctrl = O.EditController(prompts, swap, {"default_": cross}, self_, tokenizer,
                            blend_words=((blend[0],), (blend[1],)), eq_params=eq)
    assert ctrl.num_att_layers == int(golden[f"seq/{name}/num_att_layers"])
    ws = _mini_unet_weights(cfg_id)
    ctx = np.repeat(spec.text_embeddings(cfg_id), spec.F, axis=0)
    flips = 0
    for step in range(spec.NUM_STEPS_SIM):
        for b in range(16):
            xc, xt = spec.block_inputs(cfg_id, step, b)
            oc, _ = O.hooked_forward(xc, ctx, ws[b]["attn2"], spec.HEADS, ctrl, spec.PLACES[b])
            ot, _ = O.hooked_forward(xt, None, ws[b]["attn_temp"], spec.HEADS, ctrl, spec.PLACES[b])
            key = f"seq/{name}/out/{step}/{b}/cross"
            if key in golden.files:
                np.testing.assert_allclose(oc, golden[key], rtol=2e-4, atol=6e-5)
            key = f"seq/{name}/out/{step}/{b}/temp"
            if key in golden.files:
                np.testing.assert_allclose(ot, golden[key], rtol=2e-4, atol=6e-5)
        lat = spec.latents_in(cfg_id, step)
        res = ctrl.step_callback(lat.copy())
        if step in spec.LB_SAVE_STEPS:
            lb = ctrl.local_blend
            maps = ctrl.attention_store["down_cross"][2:4] + ctrl.attention_store["up_cross"][:3]
            maps = np.concatenate([m.reshape(2, -1, 8, 16, 16, 77) for m in maps], axis=2)
            wm = lb.word_maps(maps, lb.alpha_layers)
            np.testing.assert_allclose(wm, golden[f"seq/{name}/lbmaps/{step}"], rtol=1e-4)
            mask = lb.get_mask(maps, lb.alpha_layers, True)
            ref_mask = golden[f"seq/{name}/lbmask/{step}"]
            flips += int((mask != ref_mask).sum())
            same = np.broadcast_to((mask == ref_mask)[:, None], res.shape)
            np.testing.assert_array_equal(res[same], golden[f"seq/{name}/lb/{step}"][same])
            # LocalBlend(substruct_words=...): blend mask & ~(no-pool substruct mask) (run_videop2p.py:149-151)
            sw = spec.SUBSTRUCT[name]
            lbs = O.LocalBlend(prompts, ((blend[0],), (blend[1],)), tokenizer, substruct_words=((sw,), (sw,)))
            lbs.counter = lbs.start_blend
            np.testing.assert_array_equal(lbs(lat.copy(), ctrl.attention_store), golden[f"seq/{name}/lbsub/{step}"])
    assert flips == 0
    assert ctrl.cur_step == int(golden[f"seq/{name}/final_step"])
    assert ctrl.local_blend.counter == int(golden[f"seq/{name}/lb_counter"])
    assert len(ctrl.attention_store["down_cross"]) == int(golden[f"seq/{name}/store_len_down_cross"])
    assert len(ctrl.attention_store["up_self"]) == int(golden[f"seq/{name}/store_len_up_self"])


def test_ddim(golden):
    d = O.DDIM()
    np.testing.assert_array_equal(d.set_timesteps(50), golden["ddim/timesteps"])
    np.testing.assert_array_equal(d.alphas_cumprod, golden["ddim/alphas_cumprod"])
    assert d.final_alpha_cumprod == golden["ddim/final_alpha_cumprod"]
    g = spec.rng(21)
    eps = g.standard_normal((2, 4, spec.F, 8, 8)).astype(np.float32)
    x = g.standard_normal((2, 4, spec.F, 8, 8)).astype(np.float32)
    for t in spec.DDIM_PROBE_T:
        np.testing.assert_array_equal(d.step(eps, t, x), golden[f"ddim/step/{t}"])
        np.testing.assert_array_equal(d.next_step(eps, t, x), golden[f"ddim/next_step/{t}"])
        np.testing.assert_array_equal(d.prev_step(eps, t, x), golden[f"ddim/prev_step/{t}"])
