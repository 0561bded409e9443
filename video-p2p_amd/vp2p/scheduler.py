"""DDIM scheduler of the P2P path (dependent_ddim.py:78-341 with run_videop2p.py:30 arguments and
the pipeline's steps_offset=1 patch, pipeline_tuneavideo.py:61-73), plus the float32 constants
the fused step kernel needs.  eta = 0 only on the fused path (the reference default; eta > 0 and
the dependent-noise sampler are out of scope)."""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional, Tuple

import numpy as np
import torch


@dataclass
class DDIMSchedulerOutput:
    prev_sample: torch.Tensor
    pred_original_sample: Optional[torch.Tensor] = None


class DDIMScheduler:
    order = 1

    def __init__(self, beta_start: float = 0.00085, beta_end: float = 0.012, beta_schedule: str = "scaled_linear",
                 num_train_timesteps: int = 1000, clip_sample: bool = False, set_alpha_to_one: bool = False,
                 steps_offset: int = 1, prediction_type: str = "epsilon"):
        if beta_schedule == "scaled_linear":
            self.betas = torch.linspace(beta_start ** 0.5, beta_end ** 0.5, num_train_timesteps, dtype=torch.float32) ** 2
        elif beta_schedule == "linear":
            self.betas = torch.linspace(beta_start, beta_end, num_train_timesteps, dtype=torch.float32)
        else:
            raise NotImplementedError(beta_schedule)
        if clip_sample or prediction_type != "epsilon":
            raise NotImplementedError("clip_sample / non-epsilon prediction are not used by the P2P path")
        self.alphas = 1.0 - self.betas
        self.alphas_cumprod = torch.cumprod(self.alphas, dim=0)
        self.final_alpha_cumprod = torch.tensor(1.0) if set_alpha_to_one else self.alphas_cumprod[0]
        self.init_noise_sigma = 1.0
        self.num_train_timesteps = num_train_timesteps
        self.steps_offset = steps_offset
        self.num_inference_steps = None
        self.timesteps = torch.from_numpy(np.arange(0, num_train_timesteps)[::-1].copy().astype(np.int64))

    def set_timesteps(self, num_inference_steps: int, device=None):
        self.num_inference_steps = num_inference_steps
        ratio = self.num_train_timesteps // num_inference_steps
        ts = (np.arange(0, num_inference_steps) * ratio).round()[::-1].copy().astype(np.int64)
        self.timesteps = torch.from_numpy(ts).to(device) + self.steps_offset

    def scale_model_input(self, sample, timestep=None):
        return sample

    def _ac(self, t: int) -> torch.Tensor:
        return self.alphas_cumprod[t] if t >= 0 else self.final_alpha_cumprod

    def step_constants(self, timestep: int) -> Tuple[float, float, float, float]:
        """(c1, c2, c3, c4) with x' = c4 * ((x - c1 e) / c2) + c3 e, each evaluated with the same
        float32 tensor ops as dependent_ddim.py:268-309 at eta = 0."""
        t = int(timestep)
        prev_t = t - self.num_train_timesteps // self.num_inference_steps
        a_t, a_prev = self.alphas_cumprod[t], self._ac(prev_t)
        beta_t = 1 - a_t
        std = 0.0 * ((1 - a_prev) / beta_t * (1 - a_t / a_prev)) ** 0.5
        return (float(beta_t ** 0.5), float(a_t ** 0.5), float((1 - a_prev - std ** 2) ** 0.5),
                float(a_prev ** 0.5))

    def next_step_constants(self, timestep: int) -> Tuple[float, float, float, float]:
        """NullInversion.next_step (run_videop2p.py:455-463)."""
        t = int(timestep)
        cur = min(t - self.num_train_timesteps // self.num_inference_steps, 999)
        a_t, a_next = self._ac(cur), self.alphas_cumprod[t]
        return (float((1 - a_t) ** 0.5), float(a_t ** 0.5), float((1 - a_next) ** 0.5), float(a_next ** 0.5))

    def prev_step_constants(self, timestep: int) -> Tuple[float, float, float, float]:
        """NullInversion.prev_step (run_videop2p.py:445-453)."""
        t = int(timestep)
        prev_t = t - self.num_train_timesteps // self.num_inference_steps
        a_t, a_prev = self.alphas_cumprod[t], self._ac(prev_t)
        return (float((1 - a_t) ** 0.5), float(a_t ** 0.5), float((1 - a_prev) ** 0.5), float(a_prev ** 0.5))

    def step(self, model_output: torch.Tensor, timestep: int, sample: torch.Tensor, eta: float = 0.0,
             return_dict: bool = True, **_):
        """Reference-compatible eta=0 step through the fused kernel (no CFG, no blend)."""
        if eta != 0.0:
            raise NotImplementedError("eta > 0 (stochastic DDIM / dependent noise) is out of scope")
        from . import ops
        out = ops.step_fused(model_output.contiguous(), sample.float().contiguous(), self.step_constants(timestep),
                             cfg=False)
        return DDIMSchedulerOutput(prev_sample=out) if return_dict else (out,)
