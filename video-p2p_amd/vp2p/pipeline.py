"""Sampling loop of the P2P edit and the DDIM inversion driver.

``VideoP2PPipeline.__call__`` follows TuneAVideoPipeline.__call__ (pipeline_tuneavideo.py:321-442):
CFG batch [uncond x P, cond x P], optional per-step null-text embeddings (``uncond_embeddings_pre``
overwrites row 0, :399-403), fast mode (source row unguided, :412-415), DDIM step and the
controller's step callback (LocalBlend).  With a vp2p controller the CFG + DDIM + LocalBlend tail
of every step is ONE kernel (``ops.step_fused``).  VAE decoding is out of scope: the pipeline
returns latents (``output_type="latent"``).

``NullInversion.ddim_loop`` / ``invert_`` follow run_videop2p.py:557-567 / :626-635 on latents
(image loading and the VAE encoder are out of scope).  Null-text optimisation (``invert``,
:580-624) needs attention backward kernels and is not implemented yet.
"""
from __future__ import annotations

from typing import List, Optional, Union

import torch

from . import ops
from .scheduler import DDIMScheduler

NUM_DDIM_STEPS = 50
GUIDANCE_SCALE = 7.5


class VideoP2PPipeline:
    def __init__(self, unet, scheduler: Optional[DDIMScheduler] = None, tokenizer=None, text_encoder=None):
        self.unet = unet
        self.scheduler = scheduler or DDIMScheduler()
        self.tokenizer = tokenizer
        self.text_encoder = text_encoder

    @property
    def device(self):
        return next(self.unet.parameters()).device

    @torch.no_grad()
    def encode_prompt(self, prompts: List[str]) -> torch.Tensor:
        """[uncond x P, cond x P] text embeddings (pipeline_tuneavideo.py:150-237)."""
        if self.text_encoder is None or self.tokenizer is None:
            raise ValueError("pass text_embeddings= or give the pipeline a tokenizer and text_encoder")
        dev = self.device
        ids = self.tokenizer(prompts, padding="max_length", max_length=self.tokenizer.model_max_length,
                             truncation=True, return_tensors="pt").input_ids.to(dev)
        cond = self.text_encoder(ids)[0]
        unc_ids = self.tokenizer([""] * len(prompts), padding="max_length",
                                 max_length=self.tokenizer.model_max_length, return_tensors="pt").input_ids.to(dev)
        unc = self.text_encoder(unc_ids)[0]
        return torch.cat([unc, cond])

    @torch.no_grad()
    def __call__(self, prompt: Union[str, List[str]], video_length: int, height: int = 512, width: int = 512,
                 num_inference_steps: int = NUM_DDIM_STEPS, guidance_scale: float = GUIDANCE_SCALE,
                 latents: Optional[torch.Tensor] = None, uncond_embeddings_pre=None, controller=None,
                 fast: bool = False, eta: float = 0.0, text_embeddings: Optional[torch.Tensor] = None,
                 generator=None, output_type: str = "latent", **kwargs):
        if eta != 0.0:
            raise NotImplementedError("eta > 0 is out of scope (deterministic DDIM only)")
        if output_type != "latent":
            raise NotImplementedError("VAE decoding is out of scope; use output_type='latent'")
        prompts = [prompt] if isinstance(prompt, str) else list(prompt)
        P = len(prompts)
        dev = self.device
        emb = (self.encode_prompt(prompts) if text_embeddings is None else text_embeddings).to(dev).clone()
        self.scheduler.set_timesteps(num_inference_steps)
        shape = (P, self.unet.in_channels, video_length, height // 8, width // 8)
        if latents is None:
            latents = torch.randn(shape, generator=generator, dtype=torch.float32).to(dev)
        lat = latents.to(dev, torch.float32).expand(shape).contiguous() * self.scheduler.init_noise_sigma
        fused = controller is not None and hasattr(controller, "blend_plan")
        lb_th = 0.3
        if fused and controller.local_blend is not None:
            lb_th = controller.local_blend.th[0]
        for i, t in enumerate(self.scheduler.timesteps.tolist()):
            if uncond_embeddings_pre is not None:
                emb[0] = uncond_embeddings_pre[i]
            model_in = torch.cat([lat, lat])
            noise = self.unet(model_in, t, encoder_hidden_states=emb).sample.contiguous()
            if fused or controller is None:
                acc = controller.blend_plan() if fused else None
                lat = ops.step_fused(noise, lat, self.scheduler.step_constants(t), guidance_scale, cfg=True,
                                     fast=fast, lb_acc=acc, lb_count=40.0, lb_th=lb_th)
            else:  # foreign controller: reference order, step_callback on the new latents
                u, c = noise.float().chunk(2)
                e = u + guidance_scale * (c - u)
                if fast:
                    e[0] = c[0]
                lat = self.scheduler.step(e.contiguous(), t, lat).prev_sample
                lat = controller.step_callback(lat).to(dev, torch.float32)
        return lat


class NullInversion:
    """run_videop2p.py:443-648 on latents."""

    def __init__(self, model: VideoP2PPipeline, num_ddim_steps: int = NUM_DDIM_STEPS):
        self.model = model
        self.num_ddim_steps = num_ddim_steps
        self.model.scheduler.set_timesteps(num_ddim_steps)
        self.context = None

    @property
    def scheduler(self):
        return self.model.scheduler

    def init_prompt(self, prompt: str, text_embeddings: Optional[torch.Tensor] = None):
        if text_embeddings is None:
            text_embeddings = self.model.encode_prompt([prompt])
        self.context = text_embeddings

    def next_step(self, model_output, timestep, sample):
        return ops.step_fused(model_output.contiguous(), sample.float().contiguous(),
                              self.scheduler.next_step_constants(timestep), cfg=False)

    def prev_step(self, model_output, timestep, sample):
        return ops.step_fused(model_output.contiguous(), sample.float().contiguous(),
                              self.scheduler.prev_step_constants(timestep), cfg=False)

    @torch.no_grad()
    def ddim_loop(self, latent: torch.Tensor):
        uncond, cond = self.context.chunk(2)
        all_latent = [latent]
        latent = latent.clone().float()
        ts = self.scheduler.timesteps.tolist()
        for i in range(self.num_ddim_steps):
            t = ts[len(ts) - i - 1]
            noise = self.model.unet(latent, t, encoder_hidden_states=cond).sample
            latent = self.next_step(noise, t, latent)
            all_latent.append(latent)
        return all_latent

    @torch.no_grad()
    def invert_(self, latent: torch.Tensor, prompt: str, text_embeddings: Optional[torch.Tensor] = None):
        """Fast mode (run_videop2p.py:626-635): DDIM inversion only; returns (latents list, x_T, None)."""
        self.init_prompt(prompt, text_embeddings)
        lats = self.ddim_loop(latent)
        return lats, lats[-1], None

    def invert(self, *a, **k):
        raise NotImplementedError("null-text optimisation needs attention backward kernels (SURVEY §8(f) rank 2)")
