"""P2P attention controllers with the reference's public surface (run_videop2p.py:129-410).

Same class names, constructor arguments, counters and call protocol as the reference:
``controller(attn, is_cross, place_in_unet)``, ``step_callback(x_t)``, ``between_steps()``,
``reset()``, fields ``cur_step`` / ``cur_att_layer`` / ``num_att_layers`` and, for edits,
``batch_size``, ``cross_replace_alpha``, ``num_self_replace``, ``local_blend``, ``mapper``,
``alphas``, ``equalizer``, ``prev_controller``, ``attention_store``, ``step_store``.

Two execution paths share that state:

* **fused** (what ``register_attention_control`` uses for these classes): the attention kernels apply
  the edit inside their softmax epilogue.  Per hooked layer the forward asks ``fused_begin`` what
  to do (edit on/off, self-replace on/off, accumulate the LocalBlend reduction, store maps),
  launches one kernel, then ``fused_end`` advances the counters exactly as ``__call__`` would.
  No probability tensor is materialised unless ``store_maps`` is set.
* **generic** (``__call__`` on a materialised ``attn``): the reference semantics on device tensors,
  used for foreign controllers and for debugging.

LocalBlend only ever reads the step-summed, word-weighted cross maps of the res-16 layers
(run_videop2p.py:131-146), so the fused path keeps exactly that reduction
(``AttentionMaps.lb_acc``: (prompts, frames, 16*16) fp32) instead of every stored map.
"""
from __future__ import annotations

import abc
from typing import Dict, List, Optional, Sequence, Tuple, Union

import torch

from . import prompt_align as pa

NUM_DDIM_STEPS = 50
MAX_NUM_WORDS = 77
LOW_RESOURCE = False
STORE_MAX_TOKENS = 32 ** 2                     # run_videop2p.py:257, 294
LB_SELECT = {"down": (2, 3), "up": (0, 1, 2)}  # attention_store["down_cross"][2:4] + ["up_cross"][:3]
LB_HW = (16, 16)                               # LocalBlend hard-codes 8 heads x 16 x 16 (:146)


class AttentionMaps(dict):
    """``attention_store`` dict (keys down/mid/up x cross/self) plus the fused LocalBlend sum."""

    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        self.lb_acc: Optional[torch.Tensor] = None
        self.lb_layers_per_step = 0

    @staticmethod
    def empty() -> "AttentionMaps":
        return AttentionMaps({"down_cross": [], "mid_cross": [], "up_cross": [],
                              "down_self": [], "mid_self": [], "up_self": []})


class LayerCall:
    """What the fused kernel must do for one hooked layer call (built by ``fused_begin``)."""
    __slots__ = ("edit", "step", "plan", "self_replace", "lb_acc", "store", "prompts", "cond_only")

    def __init__(self):
        self.cond_only = False     # set by the hook: the batch is only the conditional half (CFG split)
        self.edit = False
        self.step = 0
        self.plan = None
        self.self_replace = False
        self.lb_acc = None
        self.store = False
        self.prompts = 0


class LocalBlend:
    """run_videop2p.py:129-180.  ``words`` per prompt; mask from step-summed res-16 cross maps."""

    def __init__(self, prompts: List[str], words, tokenizer=None, substruct_words=None,
                 start_blend: float = 0.2, th=(0.3, 0.3), num_steps: int = NUM_DDIM_STEPS):
        if tokenizer is None:
            raise ValueError("LocalBlend needs the tokenizer (the reference closes over main's)")
        self.alpha_layers = self._layers(prompts, words, tokenizer)
        self.substruct_layers = None
        if substruct_words is not None:      # run_videop2p.py:166-174
            self.substruct_layers = self._layers(prompts, substruct_words, tokenizer)
        self.start_blend = int(start_blend * num_steps)
        self.counter = 0
        self.th = th

    @staticmethod
    def _layers(prompts, words, tokenizer):
        a = torch.zeros(len(prompts), 1, 1, 1, 1, MAX_NUM_WORDS)
        for i, (prompt, ws) in enumerate(zip(prompts, words)):
            for w in ([ws] if isinstance(ws, str) else ws):
                a[i, :, :, :, :, pa.get_word_inds(prompt, w, tokenizer)] = 1
        return a

    def word_alpha(self) -> torch.Tensor:
        """Word weights the cross kernel accumulates with: (P, 77), or (2, P, 77) when
        ``substruct_words`` is set (set 1 feeds the substruct mask, run_videop2p.py:149-151)."""
        P = self.alpha_layers.shape[0]
        a = self.alpha_layers.reshape(P, MAX_NUM_WORDS)
        if self.substruct_layers is None:
            return a
        return torch.stack([a, self.substruct_layers.reshape(P, MAX_NUM_WORDS)])

    @property
    def sets(self) -> int:
        return 1 if self.substruct_layers is None else 2

    def advance(self, attention_store: AttentionMaps, required: bool = True) -> Optional[torch.Tensor]:
        """Count this step's callback (:143-144); return the LocalBlend sum if the blend fires.
        ``required=False`` (the unconditional rank of a CFG split, which never accumulates the sum):
        return None instead of raising when there is no sum."""
        self.counter += 1
        if self.counter <= self.start_blend:
            return None
        if attention_store.lb_acc is None and not required:
            return None
        if attention_store.lb_acc is None:
            raise ValueError("LocalBlend has no res-16 cross-attention maps to blend with "
                             "(the reference reshapes them to 8 heads x 16 x 16, run_videop2p.py:146)")
        return attention_store.lb_acc

    def __call__(self, x_t: torch.Tensor, attention_store: AttentionMaps, step: int = 0) -> torch.Tensor:
        acc = self.advance(attention_store)
        if acc is None:
            return x_t
        from . import ops
        P = x_t.shape[0]
        x = x_t.float().contiguous()
        # identity DDIM constants: the fused step kernel then only applies the blend
        zeros = torch.zeros_like(x)
        return ops.step_fused(zeros, x, (0.0, 1.0, 0.0, 1.0), cfg=False, lb_acc=acc, lb_hw=LB_HW,
                              lb_count=float(attention_store.lb_layers_per_step * 8), lb_th=self.th[0],
                              lb_sub_th=self.th[1])


class AttentionControl(abc.ABC):
    """run_videop2p.py:196-233."""

    def step_callback(self, x_t):
        return x_t

    def between_steps(self):
        return

    @property
    def num_uncond_att_layers(self):
        return self.num_att_layers if LOW_RESOURCE else 0

    @abc.abstractmethod
    def forward(self, attn, is_cross: bool, place_in_unet: str):
        raise NotImplementedError

    def _advance(self):
        self.cur_att_layer += 1
        if self.cur_att_layer == self.num_att_layers + self.num_uncond_att_layers:
            self.cur_att_layer = 0
            self.cur_step += 1
            self.between_steps()

    def __call__(self, attn, is_cross: bool, place_in_unet: str):
        if self.cur_att_layer >= self.num_uncond_att_layers:
            h = attn.shape[0]
            attn[h // 2:] = self.forward(attn[h // 2:], is_cross, place_in_unet)
        self._advance()
        return attn

    def reset(self):
        self.cur_step = 0
        self.cur_att_layer = 0

    def __init__(self):
        self.cur_step = 0
        self.num_att_layers = -1
        self.cur_att_layer = 0

    # -- fused protocol (default: plain attention, counters only) -----------------------------
    fused = True

    def fused_begin(self, is_cross: bool, place_in_unet: str, tokens: int, frames: int) -> LayerCall:
        return LayerCall()

    def fused_end(self, is_cross: bool, place_in_unet: str, call: LayerCall, probs=None):
        self._advance()


class EmptyControl(AttentionControl):
    def forward(self, attn, is_cross: bool, place_in_unet: str):
        return attn


class AttentionStore(AttentionControl):
    """run_videop2p.py:248-283.  ``store_maps`` keeps the full post-edit maps (N <= 32^2) like
    the reference; the fused LocalBlend sum is kept either way when a LocalBlend needs it."""

    @staticmethod
    def get_empty_store():
        return AttentionMaps.empty()

    def forward(self, attn, is_cross: bool, place_in_unet: str):
        key = f"{place_in_unet}_{'cross' if is_cross else 'self'}"
        if attn.shape[1] <= STORE_MAX_TOKENS:
            self.step_store[key].append(attn)
        return attn

    def between_steps(self):
        if len(self.attention_store) == 0 or not any(len(v) for v in self.attention_store.values()):
            lb, n = self.attention_store.lb_acc, self.attention_store.lb_layers_per_step
            self.attention_store, self.step_store = self.step_store, self.get_empty_store()
            self.attention_store.lb_acc, self.attention_store.lb_layers_per_step = lb, n
        else:
            for key in self.attention_store:
                for i in range(len(self.attention_store[key])):
                    self.attention_store[key][i] += self.step_store[key][i]
            self.step_store = self.get_empty_store()
        self._step_counts = {}

    def get_average_attention(self):
        return {key: [item / self.cur_step for item in self.attention_store[key]]
                for key in self.attention_store}

    def reset(self):
        super().reset()
        self.step_store = self.get_empty_store()
        self.attention_store = self.get_empty_store()
        self._step_counts = {}

    def __init__(self, store_maps: bool = True):
        super().__init__()
        self.store_maps = store_maps
        self.step_store = self.get_empty_store()
        self.attention_store = self.get_empty_store()
        self._step_counts: Dict[str, int] = {}

    # -- fused --------------------------------------------------------------------------------
    def _store_index(self, key: str, tokens: int) -> int:
        """Index this call's map would get in step_store[key] (-1 if not stored)."""
        if tokens > STORE_MAX_TOKENS:
            return -1
        n = self._step_counts.get(key, 0)
        self._step_counts[key] = n + 1
        return n

    def fused_begin(self, is_cross, place_in_unet, tokens, frames):
        c = LayerCall()
        c.store = self.store_maps and tokens <= STORE_MAX_TOKENS
        self._store_index(f"{place_in_unet}_{'cross' if is_cross else 'self'}", tokens)
        return c

    def fused_end(self, is_cross, place_in_unet, call, probs=None):
        if call.store and probs is not None:
            from . import frame_parallel
            lay = frame_parallel.active_layout()
            if lay is not None and lay.cfg_split and not call.cond_only:
                pass                                   # unconditional rank of a CFG split: nothing stored
            else:
                h = probs.shape[0]
                self.step_store[f"{place_in_unet}_{'cross' if is_cross else 'self'}"].append(
                    probs if call.cond_only else probs[h // 2:])
        self._advance()


class AttentionControlEdit(AttentionStore, abc.ABC):
    """run_videop2p.py:286-329."""

    def step_callback(self, x_t):
        if self.local_blend is not None:
            x_t = self.local_blend(x_t, self.attention_store, self.cur_step)
        return x_t

    def replace_self_attention(self, attn_base, att_replace, place_in_unet=None):
        if att_replace.shape[2] <= STORE_MAX_TOKENS:
            return attn_base.unsqueeze(0).expand(att_replace.shape[0], *attn_base.shape)
        return att_replace

    @abc.abstractmethod
    def replace_cross_attention(self, attn_base, att_replace):
        raise NotImplementedError

    def self_replace_active(self, frames: int) -> bool:
        return self.num_self_replace[0] <= self.cur_step < self.num_self_replace[1] and frames <= STORE_MAX_TOKENS

    def forward(self, attn, is_cross: bool, place_in_unet: str):
        super().forward(attn, is_cross, place_in_unet)
        if is_cross or (self.num_self_replace[0] <= self.cur_step < self.num_self_replace[1]):
            h = attn.shape[0] // self.batch_size
            attn = attn.reshape(self.batch_size, h, *attn.shape[1:])
            attn_base, attn_replace = attn[0], attn[1:]
            if is_cross:
                alpha_words = self.cross_replace_alpha[self.cur_step].to(attn.device)
                new = self.replace_cross_attention(attn_base, attn_replace) * alpha_words + \
                    (1 - alpha_words) * attn_replace
                attn[1:] = new
            else:
                attn[1:] = self.replace_self_attention(attn_base, attn_replace, place_in_unet)
            attn = attn.reshape(self.batch_size * h, *attn.shape[2:])
        return attn

    def __init__(self, prompts, num_steps: int,
                 cross_replace_steps: Union[float, Tuple[float, float], Dict[str, Tuple[float, float]]],
                 self_replace_steps: Union[float, Tuple[float, float]],
                 local_blend: Optional[LocalBlend], tokenizer=None, store_maps: bool = False):
        super().__init__(store_maps=store_maps)
        if tokenizer is None:
            raise ValueError("controllers need the tokenizer (the reference closes over main's)")
        self.tokenizer = tokenizer
        self.batch_size = len(prompts)
        self.cross_replace_alpha = pa.get_time_words_attention_alpha(prompts, num_steps, cross_replace_steps,
                                                                     tokenizer)
        if isinstance(self_replace_steps, float):
            self_replace_steps = 0, self_replace_steps
        self.num_self_replace = int(num_steps * self_replace_steps[0]), int(num_steps * self_replace_steps[1])
        self.local_blend = local_blend
        self._plan = None
        self._alpha_any = self.cross_replace_alpha.reshape(num_steps + 1, -1).amax(1) > 0

    # -- fused --------------------------------------------------------------------------------
    def edit_spec(self):
        """(edit_mode, reweight, mapper, refine_alpha, equalizer) of the whole controller chain."""
        raise NotImplementedError

    def plan(self, device) -> "object":
        from . import ops
        if self._plan is None or self._plan.alpha_steps.device != torch.device(device):
            mode, rew, mapper, ralpha, eq = self.edit_spec()
            lbw = self.local_blend.word_alpha() if self.local_blend is not None else None
            self._plan = ops.CrossEditPlan(self.batch_size, mode, rew,
                                           self.cross_replace_alpha.reshape(self.cross_replace_alpha.shape[0], -1),
                                           mapper=mapper, refine_alpha=ralpha, equalizer=eq,
                                           lb_word_alpha=lbw, device=device)
        return self._plan

    def fused_begin(self, is_cross, place_in_unet, tokens, frames):
        c = LayerCall()
        key = f"{place_in_unet}_{'cross' if is_cross else 'self'}"
        idx = self._store_index(key, tokens)
        c.store = self.store_maps and idx >= 0
        c.prompts = self.batch_size
        c.step = self.cur_step
        if is_cross:
            c.edit = self.cur_step < len(self._alpha_any) and bool(self._alpha_any[self.cur_step])
            if self.local_blend is not None and idx in LB_SELECT.get(place_in_unet, ()):
                if tokens != LB_HW[0] * LB_HW[1]:
                    raise ValueError(f"LocalBlend reshapes {key}[{idx}] to 16x16 but it has {tokens} tokens "
                                     "(run_videop2p.py:146)")
                c.lb_acc = True
        else:
            c.self_replace = self.self_replace_active(frames)
        return c

    def lb_buffer(self, frames: int, device) -> torch.Tensor:
        st = self.attention_store
        shape = self.lb_shape(frames)
        if st.lb_acc is None:
            st.lb_acc = torch.zeros(shape, device=device)
            st.lb_layers_per_step = len(LB_SELECT["down"]) + len(LB_SELECT["up"])
        elif tuple(st.lb_acc.shape) != shape:
            raise ValueError(f"LocalBlend sum is {tuple(st.lb_acc.shape)}, this call needs {shape}")
        return st.lb_acc

    def blend_plan(self, required: bool = True) -> Optional[torch.Tensor]:
        """Fused pipeline's replacement for ``step_callback``: the LocalBlend sum if it fires."""
        if self.local_blend is None:
            return None
        return self.local_blend.advance(self.attention_store, required)

    def blend_fires(self) -> bool:
        """Whether the NEXT step callback applies the blend (counter + 1 > start_blend, :143-144)."""
        return self.local_blend is not None and self.local_blend.counter + 1 > self.local_blend.start_blend

    def lb_shape(self, frames: int):
        shape = (self.batch_size, frames, LB_HW[0] * LB_HW[1])
        return shape if self.local_blend is None or self.local_blend.sets == 1 else (self.local_blend.sets,) + shape

    def reset(self):
        super().reset()
        if getattr(self, "local_blend", None) is not None:
            self.local_blend.counter = 0


class AttentionReplace(AttentionControlEdit):
    """run_videop2p.py:331-339: word swap through the (77 x 77) replacement mapper."""

    def replace_cross_attention(self, attn_base, att_replace):
        return torch.einsum("hpw,bwn->bhpn", attn_base, self.mapper.to(attn_base.device))

    def edit_spec(self):
        from ._lib import EDIT_REPLACE
        return EDIT_REPLACE, False, self.mapper, None, None

    def __init__(self, prompts, num_steps: int, cross_replace_steps, self_replace_steps,
                 local_blend: Optional[LocalBlend] = None, tokenizer=None, store_maps: bool = False):
        super().__init__(prompts, num_steps, cross_replace_steps, self_replace_steps, local_blend,
                         tokenizer, store_maps)
        self.mapper = pa.get_replacement_mapper(prompts, tokenizer)


class AttentionRefine(AttentionControlEdit):
    """run_videop2p.py:342-354: aligned-token refinement (new words keep their own attention)."""

    def replace_cross_attention(self, attn_base, att_replace):
        base = attn_base[:, :, self.mapper.to(attn_base.device)].permute(2, 0, 1, 3)
        a = self.alphas.to(attn_base.device)
        return base * a + att_replace * (1 - a)

    def edit_spec(self):
        from ._lib import EDIT_REFINE
        return EDIT_REFINE, False, self.mapper, self.alphas.reshape(self.alphas.shape[0], -1), None

    def __init__(self, prompts, num_steps: int, cross_replace_steps, self_replace_steps,
                 local_blend: Optional[LocalBlend] = None, tokenizer=None, store_maps: bool = False):
        super().__init__(prompts, num_steps, cross_replace_steps, self_replace_steps, local_blend,
                         tokenizer, store_maps)
        self.mapper, alphas = pa.get_refinement_mapper(prompts, tokenizer)
        self.alphas = alphas.reshape(alphas.shape[0], 1, 1, alphas.shape[1])


class AttentionReweight(AttentionControlEdit):
    """run_videop2p.py:357-369: scale chosen words' attention, optionally after another edit."""

    def replace_cross_attention(self, attn_base, att_replace):
        if self.prev_controller is not None:
            attn_base = self.prev_controller.replace_cross_attention(attn_base, att_replace)
        return attn_base[None, :, :, :] * self.equalizer.to(attn_base.device)[:, None, None, :]

    def edit_spec(self):
        from ._lib import EDIT_NONE
        if self.prev_controller is None:
            return EDIT_NONE, True, None, None, self.equalizer
        mode, _, mapper, ralpha, _ = self.prev_controller.edit_spec()
        return mode, True, mapper, ralpha, self.equalizer

    def __init__(self, prompts, num_steps: int, cross_replace_steps, self_replace_steps, equalizer,
                 local_blend: Optional[LocalBlend] = None, controller: Optional[AttentionControlEdit] = None,
                 tokenizer=None, store_maps: bool = False):
        super().__init__(prompts, num_steps, cross_replace_steps, self_replace_steps, local_blend,
                         tokenizer, store_maps)
        self.equalizer = equalizer
        self.prev_controller = controller


def get_equalizer(text: str, word_select, values, tokenizer) -> torch.Tensor:
    return pa.get_equalizer(text, word_select, values, tokenizer)


def make_controller(prompts: List[str], is_replace_controller: bool, cross_replace_steps: Dict[str, float],
                    self_replace_steps: float, blend_words=None, equilizer_params=None, mask_th=(.3, .3),
                    tokenizer=None, num_steps: int = NUM_DDIM_STEPS, store_maps: bool = False,
                    substruct_words=None) -> AttentionControlEdit:
    """run_videop2p.py:397-410 (the reference reads ``blend_words`` from main's ``blend_word``
    closure; here it is the argument).  ``substruct_words`` is passed to LocalBlend
    (run_videop2p.py:157, 166-174; the reference's factory never sets it)."""
    lb = None if blend_words is None else LocalBlend(prompts, blend_words, tokenizer, substruct_words=substruct_words,
                                                       th=mask_th, num_steps=num_steps)
    cls = AttentionReplace if is_replace_controller else AttentionRefine
    controller = cls(prompts, num_steps, cross_replace_steps=cross_replace_steps,
                     self_replace_steps=self_replace_steps, local_blend=lb, tokenizer=tokenizer,
                     store_maps=store_maps)
    if equilizer_params is not None:
        eq = get_equalizer(prompts[1], equilizer_params["words"], equilizer_params["values"], tokenizer)
        controller = AttentionReweight(prompts, num_steps, cross_replace_steps=cross_replace_steps,
                                       self_replace_steps=self_replace_steps, equalizer=eq, local_blend=lb,
                                       controller=controller, tokenizer=tokenizer, store_maps=store_maps)
    return controller
