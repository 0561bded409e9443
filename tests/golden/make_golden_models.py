"""Generate the MODEL-level golden fixtures from the reference's own model and pipeline code.

Build container only (it reads /root/reference at run time; nothing from there is copied, only
numeric outputs are saved).  Executed reference code:

* ``tuneavideo/models/attention.py`` (``FrameAttention`` :273-329, ``Transformer3DModel`` :32-137,
  ``BasicTransformerBlock`` :140-270), ``resnet.py`` (``ResnetBlock3D`` :111-205, 5-D GroupNorm),
  ``unet_blocks.py`` and ``unet.py`` (``UNet3DConditionModel`` :38-414) -- imported as the
  reference package, on top of ``diffusers_shim`` (a build-authored restatement of the
  diffusers-0.11.1 classes those files import);
* ``ptp_utils.register_attention_control`` and the controllers of ``run_videop2p.py`` (via
  ``make_golden.load_reference``, AST-extracted as for ``golden.npz``);
* ``TuneAVideoPipeline.__call__`` / ``prepare_latents`` / ``check_inputs`` /
  ``prepare_extra_step_kwargs`` (pipeline_tuneavideo.py:258-430), AST-extracted and bound to a
  stand-in pipeline object that supplies the text embeddings (CLIP is out of scope) and returns
  latents instead of VAE-decoding them; the scheduler is the reference's ``DDIMScheduler_dependent``.

Parts (``--part``, default ``models``):
  models     -> golden_models.npz: FrameAttention, Transformer3DModel (plain and hooked),
                ResnetBlock3D, and the SD-1.5-geometry UNet3D on a 16x16 latent (DummyController
                hook, and a controlled bird edit at two controller steps).  ~1 min.
  nulltext   -> golden_nulltext.npz: NullInversion.ddim_loop + null_optimization (run_videop2p.py:557-612,
                AST-extracted) on the reference UNet, 2 DDIM steps x up to 3 Adam iterations, at two
                configs (model_spec.NULLTEXT): the 256/512-channel UNet on a 32^2 latent and the
                SD-1.5 geometry on a 16^2 latent; saves every inner loss, the optimised unconditional
                embeddings and the inversion latents.  ~2 min.
  car2 | rabbit8 | penguin24l
             -> golden_edit_<part>.npz: the fast-mode P2P edit of model_spec.EDITS[part] through
                the reference pipeline loop at the SD-1.5 geometry, 512^2 (64^2 latent).  CPU-hours
                for rabbit8/penguin24l (run in the background).
"""
from __future__ import annotations

import argparse
import contextlib
import inspect
import os
import sys
import time
import types
from typing import Callable, Dict, List, Optional, Union

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import diffusers_shim  # noqa: E402
import make_golden  # noqa: E402  (load_reference, _extract, REF, MiniUNet helpers)
import model_spec as MS  # noqa: E402
import spec  # noqa: E402
from vp2p.tokenizer import SyntheticCLIPTokenizer  # noqa: E402

REF = make_golden.REF
torch.set_grad_enabled(False)


def ref_models():
    diffusers_shim.install()
    if REF not in sys.path:
        sys.path.insert(0, REF)
    import tuneavideo.models.attention as ref_attention
    import tuneavideo.models.resnet as ref_resnet
    import tuneavideo.models.unet as ref_unet
    return ref_attention, ref_resnet, ref_unet


def hook(ptp, module_tree, controller):
    """ptp_utils.register_attention_control on a bare module: it walks ``model.unet``'s children
    named down*/mid*/up*, so wrap the module as the single 'down_blocks' child."""
    class Holder(torch.nn.Module):
        def __init__(self, m):
            super().__init__()
            self.down_blocks = m

    if hasattr(module_tree, "down_blocks") and hasattr(module_tree, "up_blocks"):
        ptp.register_attention_control(types.SimpleNamespace(unet=module_tree), controller)
    else:
        ptp.register_attention_control(types.SimpleNamespace(unet=Holder(module_tree)), controller)


def part_models(ptp, ns) -> Dict[str, np.ndarray]:
    ref_attention, ref_resnet, ref_unet = ref_models()
    out: Dict[str, np.ndarray] = {}
    for name, (B, f, N, C) in MS.FA_CONFIGS.items():
        m = MS.fill_(ref_attention.FrameAttention(query_dim=C, heads=MS.HEADS, dim_head=C // MS.HEADS), 41)
        out[f"fa/{name}"] = m(torch.from_numpy(MS.fa_input(name)), video_length=f).numpy()
    for name, (B, f, h, w, C, D) in MS.T3D_CONFIGS.items():
        x, ctx = (torch.from_numpy(a) for a in MS.t3d_inputs(name))
        m = MS.fill_(ref_attention.Transformer3DModel(num_attention_heads=MS.HEADS, attention_head_dim=C // MS.HEADS,
                                                      in_channels=C, cross_attention_dim=D), 42)
        out[f"t3d/{name}/plain"] = m(x, encoder_hidden_states=ctx).sample.numpy()
        hook(ptp, m, None)            # the DummyController hook: global-max softmax (ptp_utils.py:196-234)
        out[f"t3d/{name}/hooked"] = m(x, encoder_hidden_states=ctx).sample.numpy()
    for name, (B, f, h, w, cin, cout, T) in MS.RN_CONFIGS.items():
        x, temb = (torch.from_numpy(a) for a in MS.rn_inputs(name))
        m = MS.fill_(ref_resnet.ResnetBlock3D(in_channels=cin, out_channels=cout, temb_channels=T), 43)
        out[f"rn/{name}"] = m(x, temb).numpy()

    # SD-1.5 geometry UNet3D (unet.py:42-79 defaults; cross_attention_dim 768 as in SD-1.5's config)
    unet = MS.fill_(ref_unet.UNet3DConditionModel(sample_size=64, cross_attention_dim=768), 44)
    unet.eval()
    hook(ptp, unet, None)
    sample, ctx = (torch.from_numpy(a) for a in MS.unet_small_inputs())
    t0 = time.time()
    out["unet/dummy"] = unet(sample, MS.UNET_SMALL_T, encoder_hidden_states=ctx).sample.numpy()
    print(f"[models] unet dummy forward {time.time() - t0:.1f} s", flush=True)
    # controlled forwards: the bird edit (Refine + Reweight, no LocalBlend; cross 0.8, self 0.7)
    prompts, swap, blend, eq, cross, self_ = spec.CONFIGS["bird"]
    sample4, ctx4 = (torch.from_numpy(a) for a in MS.unet_small_inputs(4))
    for s in MS.UNET_EDIT_STEPS:
        ns["x_t"] = torch.zeros(1, 4, MS.UNET_SMALL[1], MS.UNET_SMALL[2], MS.UNET_SMALL[3])
        ns["blend_word"] = None
        ctrl = ns["make_controller"](prompts, swap, {"default_": cross}, self_, None, eq)
        hook(ptp, unet, ctrl)
        ctrl.cur_step = s
        out[f"unet/bird/{s}"] = unet(sample4, MS.UNET_SMALL_T, encoder_hidden_states=ctx4).sample.numpy()
        out[f"unet/bird/{s}/layers"] = np.array(ctrl.num_att_layers)
    return out


# -- end-to-end edits through the reference pipeline loop -----------------------------------------
def ref_pipeline_call(make_scheduler):
    from einops import rearrange, repeat
    nsp = dict(torch=torch, np=np, inspect=inspect, Union=Union, List=List, Optional=Optional, Callable=Callable,
               rearrange=rearrange, repeat=repeat)
    exec(make_golden._extract(os.path.join(REF, "tuneavideo", "pipelines", "pipeline_tuneavideo.py"),
                              ["__call__", "prepare_latents", "check_inputs", "prepare_extra_step_kwargs"],
                              inside="TuneAVideoPipeline", strip_decorators=True), nsp)

    class Bar:
        def update(self, *a):
            pass

    class Pipe:
        """The attributes TuneAVideoPipeline.__call__ reads; CLIP and the VAE are out of scope."""
        vae_scale_factor = 8
        _execution_device = torch.device("cpu")

        def __init__(self, unet, emb):
            self.unet, self.emb = unet, emb
            self.scheduler = make_scheduler()
            self.scheduler.order = 1

        def _encode_prompt(self, prompt, device, num_videos_per_prompt, do_cfg, negative_prompt):
            return self.emb.clone()

        def progress_bar(self, total=None):
            return contextlib.nullcontext(Bar())

        def decode_latents(self, latents):
            return latents.numpy()

    for k in ("__call__", "prepare_latents", "check_inputs", "prepare_extra_step_kwargs"):
        setattr(Pipe, k, nsp[k])
    return Pipe


class _Stop(Exception):
    pass


def part_edit(name, ptp, ns, make_scheduler, threads, tok) -> Dict[str, np.ndarray]:
    from vp2p.unet3d import UNet3DConditionModel, init_random_
    edit, f, steps, save = MS.EDITS[name]
    prompts, swap, blend, eq, cross, self_ = spec.CONFIGS[edit]
    _, _, ref_unet = ref_models()
    torch.set_num_threads(threads)
    # the bench's weights with the res-16 attn2 q/k tied (model_spec.edit_state: localised blend maps)
    sd = MS.edit_state(init_random_(UNet3DConditionModel(), seed=0).state_dict())
    unet = ref_unet.UNet3DConditionModel(sample_size=64, cross_attention_dim=768)
    unet.load_state_dict(sd, strict=True)
    del sd
    unet.eval()
    # FrameAttention materialises (B*f*heads, 4096, 4096) scores without xformers: use the
    # reference's own attention slicing (unet.py:210-273; attention.py:319-322), one slab at a time
    unet.set_attention_slice(1)
    # the blend words' token indices from the REFERENCE's get_word_inds (ptp_utils.py:258-276)
    inp = MS.edit_inputs(name, [ptp.get_word_inds(p, w, tok) for p, w in zip(prompts, blend)])
    x_t = torch.from_numpy(inp["x_t"])
    ns["x_t"] = x_t                      # LocalBlend's closure (run_videop2p.py:136)
    ns["blend_word"] = ((blend[0],), (blend[1],))
    ctrl = ns["make_controller"](prompts, swap, {"default_": cross}, self_, ns["blend_word"], eq)
    hook(ptp, unet, ctrl)
    Pipe = ref_pipeline_call(make_scheduler)
    pipe = Pipe(unet, torch.from_numpy(inp["emb"]))
    out: Dict[str, np.ndarray] = {}
    t0 = time.time()

    def callback(i, t, latents):
        print(f"[{name}] step {i} (t={int(t)}) done at {time.time() - t0:.0f} s", flush=True)
        if i in save:
            out[f"latents/{i}"] = latents.numpy().copy()
            lb = ctrl.local_blend
            if lb.counter > lb.start_blend:     # the mask this step's callback applied
                maps = ctrl.attention_store["down_cross"][2:4] + ctrl.attention_store["up_cross"][:3]
                maps = torch.cat([m.reshape(lb.alpha_layers.shape[0], -1, 8, 16, 16, 77) for m in maps], dim=2)
                mask = lb.get_mask(maps, lb.alpha_layers, True).numpy().astype(bool)
                frac = mask.reshape(mask.shape[0], -1).mean(1)
                print(f"[{name}] step {i} mask true fraction per prompt {frac.round(3).tolist()}", flush=True)
                out[f"mask_frac/{i}"] = frac
                if not ((frac >= 0.05) & (frac <= 0.95)).all():
                    # the blend's maps are summed over steps, so the mask widens as the edit goes on;
                    # a mask that is (nearly) all True pins nothing: keep only the fraction.  The first
                    # blend step's mask must be non-trivial, or the fixture pins LocalBlend not at all.
                    if not any(k.startswith("mask/") for k in out):
                        raise RuntimeError(f"step {i}: LocalBlend mask true fraction {frac} outside [0.05, 0.95] "
                                           "-- the end-to-end mask pin would be vacuous")
                    print(f"[{name}] step {i}: mask not saved (true fraction outside [0.05, 0.95])", flush=True)
                else:
                    out[f"mask/{i}"] = np.packbits(mask)
        if i == steps - 1:
            raise _Stop

    try:
        pipe(prompts, f, latents=x_t, controller=ctrl, fast=True, num_inference_steps=50, guidance_scale=7.5,
             callback=callback, callback_steps=1, return_dict=False)
    except _Stop:
        pass
    out["steps_run"] = np.array(steps)
    out["cur_step"] = np.array(ctrl.cur_step)
    out["lb_counter"] = np.array(ctrl.local_blend.counter)
    return out


def part_nulltext(ptp, ns, make_scheduler) -> Dict[str, np.ndarray]:
    """The reference's own null-text optimisation (run_videop2p.py:580-612) with autograd and torch's
    Adam, on the reference UNet under the DummyController hook (invert() registers None, :615-616)."""
    from vp2p.unet3d import UNet3DConditionModel, init_random_
    _, _, ref_unet = ref_models()
    out: Dict[str, np.ndarray] = {}
    losses: List[float] = []

    class RecordingF:
        """nnf with mse_loss recording each inner loss (the reference keeps it in a local)."""
        def __getattr__(self, k):
            return getattr(torch.nn.functional, k)

        @staticmethod
        def mse_loss(a, b):
            loss = torch.nn.functional.mse_loss(a, b)
            losses.append(float(loss))
            return loss

    ns["nnf"] = RecordingF()
    ns["Adam"] = torch.optim.Adam
    ns["GUIDANCE_SCALE"] = 7.5
    ns["DDIMScheduler"] = lambda **kw: None      # built and discarded by NullInversion.__init__ (:637-638)
    for name, (cfg, std, x_shape, steps, inner) in MS.NULLTEXT.items():
        losses.clear()
        sd = init_random_(UNet3DConditionModel(**cfg), seed=0, std=std).state_dict()
        unet = ref_unet.UNet3DConditionModel(sample_size=64, **cfg)
        unet.load_state_dict(sd, strict=True)
        unet.eval()
        unet.requires_grad_(False)
        hook(ptp, unet, None)
        ns["NUM_DDIM_STEPS"] = steps
        model = types.SimpleNamespace(unet=unet, scheduler=make_scheduler(), tokenizer=None)
        ni = ns["NullInversion"](model)
        x0, ctx = (torch.from_numpy(a) for a in MS.nulltext_inputs(name))
        ni.context = ctx
        t0 = time.time()
        with torch.no_grad():
            lats = ni.ddim_loop(x0)
        with torch.enable_grad():
            unc = ni.null_optimization(lats, inner, 1e-5)
        print(f"[nulltext/{name}] {len(losses)} inner iterations, {time.time() - t0:.0f} s, losses {losses}", flush=True)
        out[f"{name}/losses"] = np.array(losses, np.float64)
        out[f"{name}/uncond"] = torch.cat(unc).numpy()
        out[f"{name}/latents"] = torch.stack(lats).numpy()
    ns["NUM_DDIM_STEPS"] = 50
    ns["nnf"] = torch.nn.functional
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--part", default="models", choices=["models", "nulltext"] + sorted(MS.EDITS))
    ap.add_argument("--threads", type=int, default=torch.get_num_threads())
    args = ap.parse_args()
    tok = SyntheticCLIPTokenizer()
    _, ptp, ns, make_scheduler = make_golden.load_reference(tok)
    bad = make_golden.guard_finite(ns)
    if args.part == "models":
        out = part_models(ptp, ns)
        path = os.path.join(HERE, "golden_models.npz")
    elif args.part == "nulltext":
        out = part_nulltext(ptp, ns, make_scheduler)
        path = os.path.join(HERE, "golden_nulltext.npz")
    else:
        out = part_edit(args.part, ptp, ns, make_scheduler, args.threads, tok)
        path = os.path.join(HERE, f"golden_edit_{args.part}.npz")
    if bad:
        raise RuntimeError(f"{len(bad)} hooked calls left the finite regime: {bad[:5]}")
    nonfinite = [k for k, v in out.items() if v.dtype.kind == "f" and not np.isfinite(v).all()]
    if nonfinite:
        raise RuntimeError(f"non-finite reference outputs: {nonfinite[:5]}")
    np.savez_compressed(path, **out)
    print(f"wrote {path}: {len(out)} arrays, {os.path.getsize(path) / 1e6:.2f} MB")


if __name__ == "__main__":
    main()
