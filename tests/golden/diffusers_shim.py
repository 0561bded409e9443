"""Build-authored stand-in for the parts of diffusers==0.11.1 that tuneavideo/models/*.py import.

TEST INFRASTRUCTURE ONLY (used by ``make_golden.py`` in the build container).  diffusers is not
installed here and there is no network (SURVEY §8(c), row "tuneavideo/models/*"), so the
reference's own model files -- FrameAttention's first-frame K/V gather, the 5-D GroupNorm of
ResnetBlock3D, the '(b f) d c -> (b d) f c' temporal rearrange, the block wiring of
unet_blocks.py / unet.py -- are executed against this restatement of the 0.11.1 classes they
build on.  What this file restates (and what therefore stays *parity unpinned* against the real
library):

* ``diffusers.models.attention.CrossAttention`` (0.11.1): bias-free q/k/v, ``to_out = [Linear,
  Dropout]``, scale = dim_head^-0.5, ``reshape_heads_to_batch_dim`` = (b, n, h*d) -> (b*h, n, d)
  with the batch outer, ``_attention`` = baddbmm(beta=0, alpha=scale) -> softmax -> bmm.
* ``FeedForward`` (GEGLU, mult 4), ``GEGLU`` (proj -> chunk(2) -> a * gelu(g)), ``AdaLayerNorm``.
* ``diffusers.models.embeddings.Timesteps`` / ``TimestepEmbedding`` / ``get_timestep_embedding``.
* ``ConfigMixin`` / ``register_to_config`` / ``ModelMixin`` / ``BaseOutput`` (bookkeeping only).

Nothing here is imported by the product package.
"""
from __future__ import annotations

import functools
import inspect
import math
import sys
import types
from collections import OrderedDict

import torch
import torch.nn.functional as F
from torch import nn


# -- configuration_utils / modeling_utils / utils --------------------------------------------------
class _Config(OrderedDict):
    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e


class ConfigMixin:
    config_name = "config.json"


def register_to_config(init):
    """0.11.1 semantics: every init argument (defaults included) is recorded in ``self.config`` AND
    set as an attribute BEFORE the wrapped ``__init__`` runs (that is how pipelines read
    ``unet.in_channels``)."""
    sig = inspect.signature(init)

    @functools.wraps(init)
    def wrapper(self, *args, **kwargs):
        bound = sig.bind(self, *args, **kwargs)
        bound.apply_defaults()
        cfg = _Config((k, v) for k, v in bound.arguments.items() if k not in ("self", "kwargs"))
        for k, v in cfg.items():
            object.__setattr__(self, k, v)
        object.__setattr__(self, "_internal_dict", cfg)
        init(self, *args, **kwargs)

    return wrapper


class ModelMixin(nn.Module):
    @property
    def config(self):
        return self.__dict__["_internal_dict"]

    @property
    def dtype(self):
        return next(self.parameters()).dtype

    @property
    def device(self):
        return next(self.parameters()).device


class BaseOutput:
    def __getitem__(self, i):
        if isinstance(i, str):
            return getattr(self, i)
        return tuple(getattr(self, k) for k in self.__dataclass_fields__)[i]


class _Logger:
    def info(self, *a, **k):
        pass

    warning = warn = debug = info


def is_xformers_available() -> bool:
    return False


# -- models.embeddings ----------------------------------------------------------------------------
def get_timestep_embedding(timesteps, embedding_dim, flip_sin_to_cos=False, downscale_freq_shift=1,
                           scale=1, max_period=10000):
    half_dim = embedding_dim // 2
    exponent = -math.log(max_period) * torch.arange(0, half_dim, dtype=torch.float32, device=timesteps.device)
    exponent = exponent / (half_dim - downscale_freq_shift)
    emb = torch.exp(exponent)
    emb = timesteps[:, None].float() * emb[None, :]
    emb = scale * emb
    emb = torch.cat([torch.sin(emb), torch.cos(emb)], dim=-1)
    if flip_sin_to_cos:
        emb = torch.cat([emb[:, half_dim:], emb[:, :half_dim]], dim=-1)
    if embedding_dim % 2 == 1:
        emb = F.pad(emb, (0, 1, 0, 0))
    return emb


class TimestepEmbedding(nn.Module):
    def __init__(self, in_channels: int, time_embed_dim: int, act_fn: str = "silu", out_dim: int = None):
        super().__init__()
        self.linear_1 = nn.Linear(in_channels, time_embed_dim)
        self.act = nn.SiLU() if act_fn == "silu" else None
        self.linear_2 = nn.Linear(time_embed_dim, out_dim if out_dim is not None else time_embed_dim)

    def forward(self, sample):
        sample = self.linear_1(sample)
        if self.act is not None:
            sample = self.act(sample)
        return self.linear_2(sample)


class Timesteps(nn.Module):
    def __init__(self, num_channels: int, flip_sin_to_cos: bool, downscale_freq_shift: float):
        super().__init__()
        self.num_channels = num_channels
        self.flip_sin_to_cos = flip_sin_to_cos
        self.downscale_freq_shift = downscale_freq_shift

    def forward(self, timesteps):
        return get_timestep_embedding(timesteps, self.num_channels, flip_sin_to_cos=self.flip_sin_to_cos,
                                      downscale_freq_shift=self.downscale_freq_shift)


# -- models.attention -----------------------------------------------------------------------------
class CrossAttention(nn.Module):
    def __init__(self, query_dim: int, cross_attention_dim=None, heads: int = 8, dim_head: int = 64,
                 dropout: float = 0.0, bias=False, upcast_attention: bool = False, upcast_softmax: bool = False,
                 added_kv_proj_dim=None, norm_num_groups=None):
        super().__init__()
        inner_dim = dim_head * heads
        cross_attention_dim = cross_attention_dim if cross_attention_dim is not None else query_dim
        self.upcast_attention = upcast_attention
        self.upcast_softmax = upcast_softmax
        self.scale = dim_head ** -0.5
        self.heads = heads
        self.sliceable_head_dim = heads
        self._slice_size = None
        self._use_memory_efficient_attention_xformers = False
        self.added_kv_proj_dim = added_kv_proj_dim
        self.group_norm = (nn.GroupNorm(num_channels=inner_dim, num_groups=norm_num_groups, eps=1e-5, affine=True)
                           if norm_num_groups is not None else None)
        self.to_q = nn.Linear(query_dim, inner_dim, bias=bias)
        self.to_k = nn.Linear(cross_attention_dim, inner_dim, bias=bias)
        self.to_v = nn.Linear(cross_attention_dim, inner_dim, bias=bias)
        self.to_out = nn.ModuleList([nn.Linear(inner_dim, query_dim), nn.Dropout(dropout)])

    def reshape_heads_to_batch_dim(self, tensor):
        batch_size, seq_len, dim = tensor.shape
        head_size = self.heads
        tensor = tensor.reshape(batch_size, seq_len, head_size, dim // head_size)
        return tensor.permute(0, 2, 1, 3).reshape(batch_size * head_size, seq_len, dim // head_size)

    def reshape_batch_dim_to_heads(self, tensor):
        batch_size, seq_len, dim = tensor.shape
        head_size = self.heads
        tensor = tensor.reshape(batch_size // head_size, head_size, seq_len, dim)
        return tensor.permute(0, 2, 1, 3).reshape(batch_size // head_size, seq_len, dim * head_size)

    def set_attention_slice(self, slice_size):
        self._slice_size = slice_size

    def forward(self, hidden_states, encoder_hidden_states=None, attention_mask=None):
        if self.group_norm is not None:
            hidden_states = self.group_norm(hidden_states.transpose(1, 2)).transpose(1, 2)
        query = self.reshape_heads_to_batch_dim(self.to_q(hidden_states))
        ctx = encoder_hidden_states if encoder_hidden_states is not None else hidden_states
        key = self.reshape_heads_to_batch_dim(self.to_k(ctx))
        value = self.reshape_heads_to_batch_dim(self.to_v(ctx))
        if attention_mask is not None:
            raise NotImplementedError("attention_mask (the UNet never passes one)")
        hidden_states = self._attention(query, key, value, attention_mask)
        return self.to_out[1](self.to_out[0](hidden_states))

    def _attention(self, query, key, value, attention_mask=None):
        if self.upcast_attention:
            query, key = query.float(), key.float()
        scores = torch.baddbmm(torch.empty(query.shape[0], query.shape[1], key.shape[1], dtype=query.dtype,
                                           device=query.device), query, key.transpose(-1, -2), beta=0,
                               alpha=self.scale)
        if attention_mask is not None:
            scores = scores + attention_mask
        if self.upcast_softmax:
            scores = scores.float()
        probs = scores.softmax(dim=-1).to(value.dtype)
        return self.reshape_batch_dim_to_heads(torch.bmm(probs, value))

    def _sliced_attention(self, query, key, value, sequence_length, dim, attention_mask):
        out = torch.zeros((query.shape[0], query.shape[1], dim // self.heads), device=query.device,
                          dtype=query.dtype)
        step = self._slice_size
        for i in range(query.shape[0] // step):
            s = slice(i * step, (i + 1) * step)
            scores = torch.baddbmm(torch.empty(step, query.shape[1], key.shape[1], dtype=query.dtype,
                                               device=query.device), query[s], key[s].transpose(-1, -2),
                                   beta=0, alpha=self.scale)
            out[s] = torch.bmm(scores.softmax(dim=-1).to(value.dtype), value[s])
        return self.reshape_batch_dim_to_heads(out)


class GEGLU(nn.Module):
    def __init__(self, dim_in: int, dim_out: int):
        super().__init__()
        self.proj = nn.Linear(dim_in, dim_out * 2)

    def forward(self, hidden_states):
        hidden_states, gate = self.proj(hidden_states).chunk(2, dim=-1)
        return hidden_states * F.gelu(gate)


class FeedForward(nn.Module):
    def __init__(self, dim: int, dim_out=None, mult: int = 4, dropout: float = 0.0, activation_fn: str = "geglu"):
        super().__init__()
        if activation_fn != "geglu":
            raise NotImplementedError(activation_fn)
        inner_dim = int(dim * mult)
        dim_out = dim_out if dim_out is not None else dim
        self.net = nn.ModuleList([GEGLU(dim, inner_dim), nn.Dropout(dropout), nn.Linear(inner_dim, dim_out)])

    def forward(self, hidden_states):
        for module in self.net:
            hidden_states = module(hidden_states)
        return hidden_states


class AdaLayerNorm(nn.Module):
    def __init__(self, embedding_dim, num_embeddings):
        super().__init__()
        self.emb = nn.Embedding(num_embeddings, embedding_dim)
        self.silu = nn.SiLU()
        self.linear = nn.Linear(embedding_dim, embedding_dim * 2)
        self.norm = nn.LayerNorm(embedding_dim, elementwise_affine=False)

    def forward(self, x, timestep):
        emb = self.linear(self.silu(self.emb(timestep)))
        scale, shift = torch.chunk(emb, 2)
        return self.norm(x) * (1 + scale) + shift


# -- install ----------------------------------------------------------------------------------------
def install() -> None:
    """Register the stand-in modules under the ``diffusers`` names the reference imports."""
    if "diffusers" in sys.modules and getattr(sys.modules["diffusers"], "_vp2p_shim", False):
        return
    mods = {}
    for name in ("diffusers", "diffusers.configuration_utils", "diffusers.modeling_utils", "diffusers.utils",
                 "diffusers.utils.import_utils", "diffusers.models", "diffusers.models.attention",
                 "diffusers.models.embeddings"):
        mods[name] = types.ModuleType(name)
    mods["diffusers"]._vp2p_shim = True
    mods["diffusers.configuration_utils"].ConfigMixin = ConfigMixin
    mods["diffusers.configuration_utils"].register_to_config = register_to_config
    mods["diffusers.modeling_utils"].ModelMixin = ModelMixin
    u = mods["diffusers.utils"]
    u.BaseOutput = BaseOutput
    u.logging = types.SimpleNamespace(get_logger=lambda name=None: _Logger())
    u.WEIGHTS_NAME = "diffusion_pytorch_model.bin"
    u.is_xformers_available = is_xformers_available
    mods["diffusers.utils.import_utils"].is_xformers_available = is_xformers_available
    a = mods["diffusers.models.attention"]
    a.CrossAttention, a.FeedForward, a.AdaLayerNorm, a.GEGLU = CrossAttention, FeedForward, AdaLayerNorm, GEGLU
    e = mods["diffusers.models.embeddings"]
    e.Timesteps, e.TimestepEmbedding, e.get_timestep_embedding = Timesteps, TimestepEmbedding, get_timestep_embedding
    for name, m in mods.items():
        if "." in name:
            parent, child = name.rsplit(".", 1)
            setattr(mods[parent], child, m)
        sys.modules[name] = m
