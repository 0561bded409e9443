"""Sampling loop of the P2P edit and the DDIM inversion driver.

``VideoP2PPipeline.__call__`` follows TuneAVideoPipeline.__call__ (pipeline_tuneavideo.py:321-442):
CFG batch [uncond x P, cond x P], optional per-step null-text embeddings (``uncond_embeddings_pre``
overwrites row 0, :399-403), fast mode (source row unguided, :412-415), DDIM step and the
controller's step callback (LocalBlend).  With a vp2p controller the CFG + DDIM + LocalBlend tail
of every step is ONE kernel (``ops.step_fused``).  ``output_type="tensor"`` decodes the edited
latents with the pipeline's VAE (``vp2p.vae``, per frame, on the GPU); the default returns latents.

``NullInversion.ddim_loop`` / ``invert_`` / ``invert`` follow run_videop2p.py:557-567 / :626-635 /
:614-624 on latents (image loading and the VAE encoder are out of scope).  ``null_optimization``
(:580-612) back-propagates through the UNet on the HIP backward kernels (``vp2p.autograd``); its
loss and dloss/du come from one kernel (K6b).
"""
from __future__ import annotations

from typing import List, Optional, Union

import torch

from . import frame_parallel, ops
from .attention import register_attention_control
from .scheduler import DDIMScheduler

NUM_DDIM_STEPS = 50
GUIDANCE_SCALE = 7.5


class VideoP2PPipeline:
    def __init__(self, unet, scheduler: Optional[DDIMScheduler] = None, tokenizer=None, text_encoder=None,
                 vae=None):
        self.unet = unet
        self.scheduler = scheduler or DDIMScheduler()
        self.tokenizer = tokenizer
        self.text_encoder = text_encoder
        self.vae = vae
        # debug / parity: when True, every fused step that applies LocalBlend writes the mask it applied
        # into ``blend_mask`` ((P, f, h, w) uint8, the reference's `mask`, run_videop2p.py:137-153);
        # ``blend_mask`` is None until the blend first fires
        self.keep_blend_mask = False
        self.blend_mask = None

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
                 generator=None, output_type: str = "latent", callback=None, callback_steps: int = 1,
                 graphs: bool = False, **kwargs):
        """``callback(i, t, latents)`` runs after every ``callback_steps``-th step's update (and
        LocalBlend), as in pipeline_tuneavideo.py:427-430.

        ``graphs=True``: every denoising step (UNet forward + the fused CFG/DDIM/LocalBlend step) is
        captured once as a HIP graph and replayed: the first call per (controller, shapes, schedule)
        captures and then replays, later calls only replay (``_GraphedEdit``).  Results are
        bit-identical to the eager loop.  Needs a vp2p controller (fused protocol) or none, one
        process (no frame sharding), no ``keep_blend_mask``."""
        if eta != 0.0:
            raise NotImplementedError("eta > 0 is out of scope (deterministic DDIM only)")
        if output_type not in ("latent", "tensor"):
            raise ValueError("output_type: 'latent' (the edited latents) or 'tensor' (decoded video in [0, 1])")
        if output_type == "tensor" and self.vae is None:
            raise ValueError("output_type='tensor' needs the pipeline's vae (vp2p.vae.AutoencoderKL)")
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
        if graphs:
            if not (fused or controller is None) or frame_parallel.active_layout() is not None \
                    or frame_parallel.active() is not None or self.keep_blend_mask:
                raise NotImplementedError("graphs=True: a vp2p controller (or none), one process, no keep_blend_mask")
            lat = self._graphed(controller, prompts, lat, emb, num_inference_steps, guidance_scale, fast,
                                uncond_embeddings_pre, callback, callback_steps)
            if output_type == "tensor":
                from .vae import decode_latents
                return decode_latents(self.vae, lat)
            return lat
        lb_th = (0.3, 0.3)
        if fused and controller.local_blend is not None:
            lb_th = controller.local_blend.th
        # CFG split (frame_parallel.EditLayout): this rank runs one half of the CFG batch; the halves
        # meet in one all-gather of the UNet output per step, exactly where the reference combines them
        lay = frame_parallel.active_layout()
        split = lay is not None and lay.cfg_split
        if split and not (fused or controller is None):
            raise NotImplementedError("a CFG-split edit needs a vp2p controller (fused protocol)")
        for i, t in enumerate(self.scheduler.timesteps.tolist()):
            if uncond_embeddings_pre is not None:
                emb[0] = uncond_embeddings_pre[i]
            if split:
                noise = self.unet(lat, t, encoder_hidden_states=lay.batch_rows(emb)).sample
                noise = lay.gather_cfg(noise)
            else:
                model_in = torch.cat([lat, lat])
                noise = self.unet(model_in, t, encoder_hidden_states=emb).sample.contiguous()
            if fused or controller is None:
                acc = None
                if fused and split:
                    fires = controller.blend_fires()
                    acc = controller.blend_plan(required=lay.half == 1)
                    if fires:
                        acc = lay.share_blend(acc, controller.lb_shape(lat.shape[2]), dev)
                elif fused:
                    acc = controller.blend_plan()
                mask = None
                if self.keep_blend_mask and acc is not None:
                    if self.blend_mask is None or tuple(self.blend_mask.shape) != (P,) + tuple(lat.shape[2:]):
                        self.blend_mask = torch.empty((P,) + tuple(lat.shape[2:]), device=dev, dtype=torch.uint8)
                    mask = self.blend_mask
                lat = ops.step_fused(noise, lat, self.scheduler.step_constants(t), guidance_scale, cfg=True,
                                     fast=fast, lb_acc=acc, lb_count=40.0, lb_th=lb_th[0], lb_sub_th=lb_th[1],
                                     mask_out=mask)
            else:  # foreign controller: reference order, step_callback on the new latents
                u, c = noise.float().chunk(2)
                e = u + guidance_scale * (c - u)
                if fast:
                    e[0] = c[0]
                lat = self.scheduler.step(e.contiguous(), t, lat).prev_sample
                lat = controller.step_callback(lat).to(dev, torch.float32)
            if callback is not None and i % callback_steps == 0:
                callback(i, t, lat)
        if output_type == "tensor":             # decode_latents (pipeline_tuneavideo.py:433-437)
            from .vae import decode_latents
            return decode_latents(self.vae, lat)
        return lat


    def _graphed(self, controller, prompts, lat0, emb0, steps, guidance, fast, uncond_pre, callback, callback_steps):
        """ONE captured edit is kept: an edit with another controller or shape replaces it, and the
        old graphs, their private memory pool and the old controller are released first (a session
        that builds a controller per edit stays bounded)."""
        key = (tuple(lat0.shape), tuple(emb0.shape), steps, float(guidance), bool(fast),
               uncond_pre is not None, str(lat0.device))
        hit = self.__dict__.get("_graph_cache")
        if hit is not None and hit[0] == key and hit[1].controller is controller:
            ge = hit[1]
        else:
            self.__dict__["_graph_cache"] = None
            del hit
            torch.cuda.synchronize(lat0.device)
            ge = _GraphedEdit(self, controller, prompts, lat0, emb0, steps, guidance, fast, uncond_pre)
            self.__dict__["_graph_cache"] = (key, ge)
        return ge.run(lat0, emb0, uncond_pre, callback, callback_steps)


class _GraphedEdit:
    """One captured edit: a HIP graph per denoising step (pipeline_tuneavideo.py:394-430 body), all
    in one private memory pool and replayed in capture order.  The per-step scalars (timestep, DDIM
    constants, the controller's step-dependent edit / self-replace / LocalBlend decisions and its
    word-alpha row) are baked into step i's graph when it is captured; the tensors a replay reads
    are static buffers refreshed by ``run``: the initial latents, the text embeddings and the
    optional per-step unconditional embeddings."""

    def __init__(self, pipe, controller, prompts, lat0, emb0, steps, guidance, fast, uncond_pre):
        self.controller = controller
        unet, sched = pipe.unet, pipe.scheduler
        dev = lat0.device
        sched.set_timesteps(steps)
        self.ts = sched.timesteps.tolist()
        P = len(prompts)
        self.lat_in = lat0.clone()
        self.emb = emb0.clone()
        self.unc = None if uncond_pre is None else torch.stack([u.reshape(self.emb[0].shape) for u in uncond_pre]).to(dev)
        t_dev = [torch.tensor([t], dtype=torch.int64, device=dev) for t in self.ts]
        fused = controller is not None
        lb_th = (0.3, 0.3)
        if fused:
            controller.plan(dev)                       # device tables built outside the capture
            if controller.local_blend is not None:
                lb_th = controller.local_blend.th
        # warm-up: one eager forward makes every lazy cache (concatenated weights, kernel attributes,
        # code objects) before the capture, then the controller starts the edit afresh
        torch.cuda.synchronize(dev)
        with torch.no_grad():
            unet(torch.cat([self.lat_in, self.lat_in]), t_dev[0], encoder_hidden_states=self.emb)
        if controller is not None:
            controller.reset()
        torch.cuda.synchronize(dev)
        self.pool = torch.cuda.graph_pool_handle()
        self.graphs, self.lats = [], []
        lat = self.lat_in
        with torch.no_grad():
            for i, t in enumerate(self.ts):
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, pool=self.pool):
                    if self.unc is not None:
                        self.emb[0].copy_(self.unc[i])
                    noise = unet(torch.cat([lat, lat]), t_dev[i], encoder_hidden_states=self.emb).sample.contiguous()
                    acc = controller.blend_plan() if fused else None
                    lat = ops.step_fused(noise, lat, sched.step_constants(t), guidance, cfg=True, fast=fast,
                                         lb_acc=acc, lb_count=40.0, lb_th=lb_th[0], lb_sub_th=lb_th[1])
                    del noise
                self.graphs.append(g)
                self.lats.append(lat)
        # buffers the replays write across steps stay referenced for the graphs' lifetime
        self.keep = [t_dev, None if controller is None else getattr(controller.attention_store, "lb_acc", None)]

    def run(self, lat0, emb0, uncond_pre, callback, callback_steps):
        if lat0.data_ptr() != self.lat_in.data_ptr():
            self.lat_in.copy_(lat0)
        self.emb.copy_(emb0)
        if uncond_pre is not None:
            self.unc.copy_(torch.stack([u.reshape(self.emb[0].shape) for u in uncond_pre]))
        for i, (g, t) in enumerate(zip(self.graphs, self.ts)):
            g.replay()
            if callback is not None and i % callback_steps == 0:
                # a copy: the graph pool's buffer is rewritten by the next replay
                callback(i, t, self.lats[i].clone())
        return self.lats[-1].clone()


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
        register_attention_control(self.model, None)
        lats = self.ddim_loop(latent)
        return lats, lats[-1], None

    @torch.no_grad()
    def get_noise_pred(self, latents, t, is_forward: bool = True, context=None):
        """run_videop2p.py:473-490: CFG over [uncond, cond] (guidance 1 forward, 7.5 backward) + step."""
        if context is None:
            context = self.context
        g = 1.0 if is_forward else GUIDANCE_SCALE
        noise = self.model.unet(torch.cat([latents] * 2), t, encoder_hidden_states=context).sample.contiguous()
        consts = self.scheduler.next_step_constants(t) if is_forward else self.scheduler.prev_step_constants(t)
        return ops.step_fused(noise, latents.float().contiguous(), consts, g, cfg=True)

    def null_optimization(self, latents, num_inner_steps: int, epsilon: float):
        """run_videop2p.py:580-612.  Per step: Adam (lr 1e-2 * (1 - i/100)) on the unconditional
        embedding for up to ``num_inner_steps`` iterations of loss = mse(prev_step(CFG noise), x_prev),
        early stop at loss < epsilon + i * 2e-5; then one guided DDIM step with the optimised
        embedding.  The UNet weights are frozen for the duration (the reference's Adam only holds the
        embedding, so its weight gradients are never used)."""
        from . import autograd
        unet = self.model.unet
        shard = frame_parallel.active()
        shard = shard if (shard is not None and shard.world > 1) else None
        was = [p.requires_grad for p in unet.parameters()]
        unet.requires_grad_(False)
        try:
            uncond, cond = self.context.chunk(2)
            out = []
            latent_cur = latents[-1]
            ts = self.scheduler.timesteps.tolist()
            self.losses = []
            for i in range(self.num_ddim_steps):
                uncond = uncond.clone().detach().float()
                uncond.requires_grad = True
                opt = torch.optim.Adam([uncond], lr=1e-2 * (1.0 - i / 100.0))
                latent_prev = latents[len(latents) - i - 2].float().contiguous()
                t = ts[i]
                consts = self.scheduler.prev_step_constants(t)
                with torch.no_grad():
                    noise_cond = unet(latent_cur, t, encoder_hidden_states=cond).sample.contiguous()
                for _ in range(num_inner_steps):
                    noise_uncond = unet(latent_cur, t, encoder_hidden_states=uncond).sample
                    loss = autograd.NullTextLoss.apply(noise_uncond, noise_cond, latent_cur.float(), latent_prev,
                                                       consts, GUIDANCE_SCALE)
                    opt.zero_grad()
                    loss.backward()
                    if shard is not None:
                        # frames sharded: the clip's loss is the mean of the ranks' equal-size MSEs, so
                        # its embedding gradient is the mean of theirs (every rank then takes the same
                        # Adam step) and the early-stop test reads the clip's loss
                        red = torch.cat([uncond.grad.reshape(-1), loss.detach().reshape(1).to(uncond.grad.dtype)])
                        shard.all_reduce_(red)
                        red /= shard.world
                        uncond.grad.copy_(red[:-1].view_as(uncond.grad))
                        loss = red[-1]
                    opt.step()
                    loss_item = loss.item()
                    self.losses.append(loss_item)
                    if loss_item < epsilon + i * 2e-5:
                        break
                out.append(uncond[:1].detach())
                with torch.no_grad():
                    context = torch.cat([uncond.to(cond.dtype), cond])
                    latent_cur = self.get_noise_pred(latent_cur, t, False, context)
            return out
        finally:
            for p, r in zip(unet.parameters(), was):
                p.requires_grad_(r)

    def invert(self, latent: torch.Tensor, prompt: str, num_inner_steps: int = 10, early_stop_epsilon: float = 1e-5,
               text_embeddings: Optional[torch.Tensor] = None):
        """Official mode (run_videop2p.py:614-624): DDIM inversion, then null-text optimisation.
        Returns (latents list, x_T, per-step unconditional embeddings)."""
        self.init_prompt(prompt, text_embeddings)
        register_attention_control(self.model, None)
        lats = self.ddim_loop(latent)
        unc = self.null_optimization(lats, num_inner_steps, early_stop_epsilon)
        return lats, lats[-1], unc
