"""CPU oracle for Video-P2P's controlled-attention path.  TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this module, and only as the checker or the timed CPU baseline; the product (``vp2p``) never
imports it and fails loudly when its HIP library is missing.

Everything here is a plain-numpy restatement of the reference algorithm, float32 throughout,
each function citing the reference file:line it follows (paths relative to the reference repo).
Parity status: PINNED — ``tests/test_oracle_golden.py`` checks every function below against
``tests/golden/golden.npz``, produced by running the reference's own code
(``tests/golden/make_golden.py``).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple, Union

import numpy as np

MAX_NUM_WORDS = 77
NUM_DDIM_STEPS = 50
STORE_MAX_TOKENS = 32 ** 2          # run_videop2p.py:257, :294


# ----------------------------------------------------------------------------------------------
# prompt / word bookkeeping
# ----------------------------------------------------------------------------------------------
def get_word_inds(text: str, word_place, tokenizer) -> np.ndarray:
    """Token positions of a word (by string or word index).  ptp_utils.py:258-276."""
    words = text.split(" ")
    if isinstance(word_place, str):
        targets = [i for i, w in enumerate(words) if w == word_place]
    elif isinstance(word_place, (int, np.integer)):
        targets = [int(word_place)]
    else:
        targets = list(word_place)
    found: List[int] = []
    if targets:
        pieces = [tokenizer.decode([t]).strip("#") for t in tokenizer.encode(text)][1:-1]
        acc = 0
        w = 0
        for i, piece in enumerate(pieces):
            acc += len(piece)
            if w in targets:
                found.append(i + 1)
            if acc >= len(words[w]):
                w += 1
                acc = 0
    return np.array(found)


def time_word_alpha(prompts: Sequence[str], num_steps: int, cross_replace_steps, tokenizer,
                    max_num_words: int = MAX_NUM_WORDS) -> np.ndarray:
    """alpha[t, p, 0, 0, w] in {0, 1}.  ptp_utils.py:279-310."""
    if not isinstance(cross_replace_steps, dict):
        cross_replace_steps = {"default_": cross_replace_steps}
    cross_replace_steps = dict(cross_replace_steps)
    cross_replace_steps.setdefault("default_", (0.0, 1.0))
    alpha = np.zeros((num_steps + 1, len(prompts) - 1, max_num_words), np.float32)

    def window(bounds, p, cols):
        if isinstance(bounds, float):
            bounds = (0, bounds)
        lo, hi = int(bounds[0] * alpha.shape[0]), int(bounds[1] * alpha.shape[0])
        alpha[:lo, p, cols] = 0
        alpha[lo:hi, p, cols] = 1
        alpha[hi:, p, cols] = 0

    everything = np.arange(max_num_words)
    for p in range(len(prompts) - 1):
        window(cross_replace_steps["default_"], p, everything)
    for key, bounds in cross_replace_steps.items():
        if key == "default_":
            continue
        for p in range(1, len(prompts)):
            inds = get_word_inds(prompts[p], key, tokenizer)
            if len(inds) > 0:
                window(bounds, p - 1, inds)
    return alpha.reshape(num_steps + 1, len(prompts) - 1, 1, 1, max_num_words)


def _needleman_wunsch(x: Sequence[int], y: Sequence[int]):
    """Global alignment, gap 0 / match 1 / mismatch -1, tie order left > up > diag.
    seq_aligner.py:34-78 (ScoreParams(0, 1, -1) at :112)."""
    nx, ny = len(x), len(y)
    score = np.zeros((nx + 1, ny + 1), np.int32)
    move = np.zeros((nx + 1, ny + 1), np.int32)
    move[0, 1:] = 1
    move[1:, 0] = 2
    move[0, 0] = 4
    for i in range(1, nx + 1):
        for j in range(1, ny + 1):
            left = score[i, j - 1]
            up = score[i - 1, j]
            diag = score[i - 1, j - 1] + (1 if x[i - 1] == y[j - 1] else -1)
            best = max(left, up, diag)
            score[i, j] = best
            move[i, j] = 1 if best == left else (2 if best == up else 3)
    return move


def _traceback_y_to_x(x, y, move) -> np.ndarray:
    """(j, i or -1) pairs in y order.  seq_aligner.py:81-106."""
    i, j = len(x), len(y)
    pairs = []
    while i > 0 or j > 0:
        m = move[i, j]
        if m == 3:
            i, j = i - 1, j - 1
            pairs.append((j, i))
        elif m == 1:
            j -= 1
            pairs.append((j, -1))
        elif m == 2:
            i -= 1
        else:
            break
    pairs.reverse()
    return np.array(pairs, dtype=np.int64).reshape(-1, 2)


def refinement_mapper(prompts: Sequence[str], tokenizer, max_len: int = MAX_NUM_WORDS):
    """(mapper int64 (P-1, 77), alphas float32 (P-1, 77)).  seq_aligner.py:109-130."""
    mappers, alphas = [], []
    x = tokenizer.encode(prompts[0])
    for p in prompts[1:]:
        y = tokenizer.encode(p)
        pairs = _traceback_y_to_x(x, y, _needleman_wunsch(x, y))
        n = pairs.shape[0]
        a = np.ones(max_len, np.float32)
        a[:n] = (pairs[:, 1] != -1).astype(np.float32)
        m = np.zeros(max_len, np.int64)
        m[:n] = pairs[:, 1]
        m[n:] = len(y) + np.arange(max_len - len(y))
        mappers.append(m)
        alphas.append(a)
    return np.stack(mappers), np.stack(alphas)


def replacement_mapper(prompts: Sequence[str], tokenizer, max_len: int = MAX_NUM_WORDS) -> np.ndarray:
    """Dense (P-1, 77, 77) float32 word-swap mapper.  seq_aligner.py:154-197."""
    out = []
    src = prompts[0]
    wx = src.split(" ")
    for tgt in prompts[1:]:
        wy = tgt.split(" ")
        if len(wx) != len(wy):
            raise ValueError("attention replacement edit can only be applied on prompts with the same "
                             f"length but prompt A has {len(wx)} words and prompt B has {len(wy)} words.")
        changed = [k for k in range(len(wy)) if wy[k] != wx[k]]
        s_inds = [get_word_inds(src, k, tokenizer) for k in changed]
        t_inds = [get_word_inds(tgt, k, tokenizer) for k in changed]
        m = np.zeros((max_len, max_len))
        i = j = c = 0
        while i < max_len and j < max_len:
            if c < len(s_inds) and s_inds[c][0] == i:
                si, ti = s_inds[c], t_inds[c]
                if len(si) == len(ti):
                    m[si, ti] = 1
                else:
                    for t in ti:
                        m[si, t] = 1 / len(ti)
                c += 1
                i += len(si)
                j += len(ti)
            elif c < len(s_inds):
                m[i, j] = 1
                i += 1
                j += 1
            else:
                m[j, j] = 1          # seq_aligner.py:183 indexes (j, j), not (i, j)
                i += 1
                j += 1
        out.append(m.astype(np.float32))
    return np.stack(out)


def equalizer(text: str, word_select, values, tokenizer) -> np.ndarray:
    """(1, 77) reweighting vector.  run_videop2p.py:372-381."""
    if isinstance(word_select, (int, str)):
        word_select = (word_select,)
    eq = np.ones((1, MAX_NUM_WORDS), np.float32)
    for w, v in zip(word_select, values):
        eq[:, get_word_inds(text, w, tokenizer)] = v
    return eq


# ----------------------------------------------------------------------------------------------
# controller (edit + store + LocalBlend)
# ----------------------------------------------------------------------------------------------
class LocalBlend:
    """run_videop2p.py:129-180 (mask from step-summed res-16 cross maps)."""

    def __init__(self, prompts, words, tokenizer, substruct_words=None, start_blend=0.2,
                 th=(0.3, 0.3), latent_hw=(64, 64)):
        self.alpha_layers = self._layers(prompts, words, tokenizer)
        self.substruct_layers = (None if substruct_words is None
                                 else self._layers(prompts, substruct_words, tokenizer))
        self.start_blend = int(start_blend * NUM_DDIM_STEPS)
        self.counter = 0
        self.th = th
        self.latent_hw = latent_hw

    @staticmethod
    def _layers(prompts, words, tokenizer):
        a = np.zeros((len(prompts), 1, 1, 1, 1, MAX_NUM_WORDS), np.float32)
        for i, (p, ws) in enumerate(zip(prompts, words)):
            if isinstance(ws, str):
                ws = [ws]
            for w in ws:
                a[i, :, :, :, :, get_word_inds(p, w, tokenizer)] = 1
        return a

    def word_maps(self, maps: np.ndarray, alpha: np.ndarray) -> np.ndarray:
        """(P, f, 40, 16, 16, 77) -> (P, f, 16, 16).  run_videop2p.py:133."""
        return (maps * alpha).sum(-1, dtype=np.float32).mean(2, dtype=np.float32)

    def mask_from_word_maps(self, m: np.ndarray, use_pool: bool) -> np.ndarray:
        """run_videop2p.py:134-140: 3x3/s1/p1 max-pool, nearest resize, per-map max, threshold, OR."""
        if use_pool:
            pad = np.pad(m, ((0, 0), (0, 0), (1, 1), (1, 1)), constant_values=-np.inf)
            h, w = m.shape[-2:]
            m = np.max(np.stack([pad[..., dy:dy + h, dx:dx + w] for dy in range(3) for dx in range(3)]),
                       axis=0)
        H, W = self.latent_hw
        h, w = m.shape[-2:]
        ys = np.floor(np.arange(H) * (h / H)).astype(np.int64)
        xs = np.floor(np.arange(W) * (w / W)).astype(np.int64)
        up = m[..., ys[:, None], xs[None, :]]
        up = up / up.max(axis=(2, 3), keepdims=True)
        mask = up > self.th[1 - int(use_pool)]
        return mask[:1] | mask

    def get_mask(self, maps, alpha, use_pool):
        return self.mask_from_word_maps(self.word_maps(maps, alpha), use_pool)

    def __call__(self, x_t: np.ndarray, attention_store: Dict[str, list]) -> np.ndarray:
        self.counter += 1
        if self.counter <= self.start_blend:
            return x_t
        maps = attention_store["down_cross"][2:4] + attention_store["up_cross"][:3]
        P = self.alpha_layers.shape[0]
        maps = np.concatenate([m.reshape(P, -1, 8, 16, 16, MAX_NUM_WORDS) for m in maps], axis=2)
        mask = self.get_mask(maps, self.alpha_layers, True)
        if self.substruct_layers is not None:
            mask = mask & ~self.get_mask(maps, self.substruct_layers, False)
        return blend_latents(x_t, mask)


def blend_latents(x_t: np.ndarray, mask: np.ndarray) -> np.ndarray:
    """x_t = x_t[:1] + mask * (x_t - x_t[:1]); mask (P, f, H, W) bool.  run_videop2p.py:152-154."""
    m = mask.astype(np.float32).reshape(mask.shape[0], 1, *mask.shape[1:])
    return (x_t[:1] + m * (x_t - x_t[:1])).astype(np.float32)


class EditController:
    """AttentionStore + AttentionControlEdit + Replace/Refine/Reweight as ``make_controller``
    assembles them.  run_videop2p.py:196-233 (counters), 248-283 (store), 286-329 (edit),
    331-369 (replace / refine / reweight), 397-410 (factory)."""

    def __init__(self, prompts, is_replace, cross_replace_steps, self_replace_steps, tokenizer,
                 blend_words=None, eq_params=None, mask_th=(0.3, 0.3), num_steps=NUM_DDIM_STEPS,
                 latent_hw=(64, 64)):
        self.batch_size = len(prompts)
        if not isinstance(cross_replace_steps, dict):
            cross_replace_steps = {"default_": cross_replace_steps}
        self.cross_replace_alpha = time_word_alpha(prompts, num_steps, cross_replace_steps, tokenizer)
        if isinstance(self_replace_steps, float):
            self_replace_steps = (0, self_replace_steps)
        self.num_self_replace = (int(num_steps * self_replace_steps[0]),
                                 int(num_steps * self_replace_steps[1]))
        self.is_replace = is_replace
        if is_replace:
            self.mapper = replacement_mapper(prompts, tokenizer)
        else:
            self.mapper, a = refinement_mapper(prompts, tokenizer)
            self.alphas = a.reshape(a.shape[0], 1, 1, a.shape[1])
        self.equalizer = (None if eq_params is None else
                          equalizer(prompts[1], eq_params["words"], eq_params["values"], tokenizer))
        self.local_blend = (None if blend_words is None else
                            LocalBlend(prompts, blend_words, tokenizer, th=mask_th, latent_hw=latent_hw))
        self.num_att_layers = 32
        self.cur_step = 0
        self.cur_att_layer = 0
        self.step_store = self._empty()
        self.attention_store: Dict[str, list] = {}

    @staticmethod
    def _empty():
        return {k: [] for k in ("down_cross", "mid_cross", "up_cross", "down_self", "mid_self", "up_self")}

    # -- edits --------------------------------------------------------------------------------
    def base_edit(self, base: np.ndarray, rep: np.ndarray) -> np.ndarray:
        """Replace (:333-334) or Refine (:344-347); base (h, N, 77), rep (P-1, h, N, 77)."""
        if self.is_replace:
            return np.einsum("hpw,bwn->bhpn", base, self.mapper).astype(np.float32)
        gathered = base[:, :, self.mapper].transpose(2, 0, 1, 3)
        return (gathered * self.alphas + rep * (1 - self.alphas)).astype(np.float32)

    def replace_cross(self, base, rep):
        r = self.base_edit(base, rep)
        if self.equalizer is not None:                     # AttentionReweight (:359-363)
            r = r[None] * self.equalizer[:, None, None, :]
            r = r.reshape(r.shape[1:]) if r.shape[0] == 1 else r
        return r

    def edit(self, attn: np.ndarray, is_cross: bool) -> np.ndarray:
        """AttentionControlEdit.forward (:304-317) on the cond half (B/2*h', N, M)."""
        if not (is_cross or self.num_self_replace[0] <= self.cur_step < self.num_self_replace[1]):
            return attn
        h = attn.shape[0] // self.batch_size
        a = attn.reshape(self.batch_size, h, *attn.shape[1:]).copy()
        base, rep = a[0], a[1:]
        if is_cross:
            al = self.cross_replace_alpha[self.cur_step]
            a[1:] = self.replace_cross(base, rep) * al + (1 - al) * rep
        elif rep.shape[2] <= STORE_MAX_TOKENS:              # replace_self_attention (:293-298)
            a[1:] = base[None]
        return a.reshape(attn.shape)

    def __call__(self, attn: np.ndarray, is_cross: bool, place: str) -> np.ndarray:
        """AttentionControl.__call__ (:212-224), LOW_RESOURCE = False: edit the cond half."""
        h = attn.shape[0]
        out = attn.copy()
        out[h // 2:] = self.edit(attn[h // 2:], is_cross)
        if out.shape[1] <= STORE_MAX_TOKENS:                 # AttentionStore.forward (:255-259)
            self.step_store[f"{place}_{'cross' if is_cross else 'self'}"].append(out[h // 2:].copy())
        self.cur_att_layer += 1
        if self.cur_att_layer == self.num_att_layers:
            self.cur_att_layer = 0
            self.cur_step += 1
            self.between_steps()
        return out

    def between_steps(self):
        """:261-268: running SUM over steps."""
        if not self.attention_store:
            self.attention_store = self.step_store
        else:
            for key, lst in self.attention_store.items():
                for i in range(len(lst)):
                    lst[i] = lst[i] + self.step_store[key][i]
        self.step_store = self._empty()

    def step_callback(self, x_t: np.ndarray) -> np.ndarray:
        """:288-291."""
        if self.local_blend is not None:
            return self.local_blend(x_t, self.attention_store)
        return x_t


# ----------------------------------------------------------------------------------------------
# attention math
# ----------------------------------------------------------------------------------------------
def heads_to_batch(t: np.ndarray, heads: int) -> np.ndarray:
    """(b, n, h*d) -> (b*h, n, d), batch-outer / head-inner (diffusers 0.11.1 CrossAttention)."""
    b, n, dim = t.shape
    return t.reshape(b, n, heads, dim // heads).transpose(0, 2, 1, 3).reshape(b * heads, n, dim // heads)


def batch_to_heads(t: np.ndarray, heads: int) -> np.ndarray:
    bh, n, d = t.shape
    return t.reshape(bh // heads, heads, n, d).transpose(0, 2, 1, 3).reshape(bh // heads, n, heads * d)


def global_max_softmax(sim: np.ndarray) -> np.ndarray:
    """exp(s - max(s_all)) / sum exp(...) with ONE max over the whole tensor.  ptp_utils.py:217."""
    e = np.exp(sim - sim.max())
    return (e / e.sum(-1, keepdims=True, dtype=np.float32)[...]).astype(np.float32)


def row_softmax(sim: np.ndarray) -> np.ndarray:
    e = np.exp(sim - sim.max(-1, keepdims=True))
    return (e / e.sum(-1, keepdims=True, dtype=np.float32)).astype(np.float32)


def hooked_probs(q: np.ndarray, k: np.ndarray, scale: float) -> np.ndarray:
    """sim = q k^T * scale, global-max softmax.  ptp_utils.py:209-217 (q,k already (b*h, n, d))."""
    sim = np.einsum("bid,bjd->bij", q, k).astype(np.float32) * np.float32(scale)
    return global_max_softmax(sim)


def hooked_forward(x: np.ndarray, context: Optional[np.ndarray], w: Dict[str, np.ndarray], heads: int,
                   controller=None, place: str = "down"):
    """The patched CrossAttention.forward.  ptp_utils.py:196-221.  w holds nn.Linear-style
    (out, in) weights to_q/to_k/to_v/to_out_w and bias to_out_b.  Returns (out, post-edit probs)."""
    is_cross = context is not None
    ctx = context if is_cross else x
    q = heads_to_batch(x @ w["to_q"].T, heads)
    k = heads_to_batch(ctx @ w["to_k"].T, heads)
    v = heads_to_batch(ctx @ w["to_v"].T, heads)
    d = q.shape[-1]
    attn = hooked_probs(q, k, d ** -0.5)
    if controller is not None:
        attn = controller(attn, is_cross, place)
    out = batch_to_heads(np.einsum("bij,bjd->bid", attn, v).astype(np.float32), heads)
    return (out @ w["to_out_w"].T + w["to_out_b"]).astype(np.float32), attn


def frame_attention(q: np.ndarray, k: np.ndarray, v: np.ndarray, video_length: int, heads: int,
                    scale: Optional[float] = None) -> np.ndarray:
    """FrameAttention core (no projections).  attention.py:282-322: K/V of frame 0 of each batch
    element serve every frame ('key[:, [0] * video_length]', :296-302); row softmax
    (diffusers ``_attention`` / xformers).  q (B*f, N, h*d); k, v (B*f, N, h*d) or (B, N, h*d)."""
    Bf, n, C = q.shape
    B = Bf // video_length
    if k.shape[0] == Bf:
        k = k.reshape(B, video_length, *k.shape[1:])[:, 0]
        v = v.reshape(B, video_length, *v.shape[1:])[:, 0]
    k = np.repeat(k, video_length, axis=0)
    v = np.repeat(v, video_length, axis=0)
    qh, kh, vh = (heads_to_batch(t, heads) for t in (q, k, v))
    s = np.float32((C // heads) ** -0.5) if scale is None else np.float32(scale)
    p = row_softmax(np.einsum("bid,bjd->bij", qh, kh).astype(np.float32) * s)
    return batch_to_heads(np.einsum("bij,bjd->bid", p, vh).astype(np.float32), heads)


def controlled_core(q: np.ndarray, k: np.ndarray, v: np.ndarray, heads: int, is_cross: bool,
                    controller=None, place: str = "down"):
    """Hooked attention after the projections: q/k/v (b, n, h*d) -> (b, n, h*d), probs."""
    qh, kh, vh = (heads_to_batch(t, heads) for t in (q, k, v))
    attn = hooked_probs(qh, kh, qh.shape[-1] ** -0.5)
    if controller is not None:
        attn = controller(attn, is_cross, place)
    out = np.einsum("bij,bjd->bid", attn, vh).astype(np.float32)
    return batch_to_heads(out, heads), attn


# ----------------------------------------------------------------------------------------------
# DDIM (eta = 0) and CFG
# ----------------------------------------------------------------------------------------------
def _torch_linspace_f32(start: float, end: float, steps: int) -> np.ndarray:
    """ATen's float32 linspace: float32 step, symmetric fill from both ends, each element one
    fused multiply-add (start + step*i / end - step*(n-1-i)), emulated exactly in float64."""
    start, end = np.float32(start), np.float32(end)
    step = np.float64((end - start) / np.float32(steps - 1))
    i = np.arange(steps, dtype=np.float64)
    lo = (np.float64(start) + step * i).astype(np.float32)
    hi = (np.float64(end) - step * (steps - 1 - i)).astype(np.float32)
    return np.where(np.arange(steps) < steps // 2, lo, hi)


class DDIM:
    """DDIMScheduler_dependent with run_videop2p.py:30 arguments and the pipeline's steps_offset=1
    patch.  dependent_ddim.py:141-170 (betas, alphas_cumprod), 196-210 (set_timesteps),
    268-309 (step, eta = 0); NullInversion.prev_step / next_step run_videop2p.py:445-463."""

    def __init__(self, beta_start=0.00085, beta_end=0.012, num_train_timesteps=1000, steps_offset=1):
        betas = _torch_linspace_f32(beta_start ** 0.5, beta_end ** 0.5, num_train_timesteps) ** 2
        self.alphas_cumprod = np.cumprod((1.0 - betas).astype(np.float64)).astype(np.float32)
        self.final_alpha_cumprod = self.alphas_cumprod[0]
        self.num_train_timesteps = num_train_timesteps
        self.steps_offset = steps_offset
        self.num_inference_steps = None

    def set_timesteps(self, n: int):
        self.num_inference_steps = n
        ratio = self.num_train_timesteps // n
        self.timesteps = (np.arange(0, n) * ratio).round()[::-1].astype(np.int64) + self.steps_offset
        return self.timesteps

    def _ac(self, t: int) -> np.float32:
        return self.alphas_cumprod[t] if t >= 0 else self.final_alpha_cumprod

    def step(self, eps: np.ndarray, t: int, x: np.ndarray) -> np.ndarray:
        prev_t = t - self.num_train_timesteps // self.num_inference_steps
        a_t, a_prev = self.alphas_cumprod[t], self._ac(prev_t)
        b_t = np.float32(1) - a_t
        x0 = (x - np.sqrt(b_t) * eps) / np.sqrt(a_t)
        direction = np.sqrt(np.float32(1) - a_prev - np.float32(0)) * eps
        return (np.sqrt(a_prev) * x0 + direction).astype(np.float32)

    def prev_step(self, eps, t, x):
        prev_t = t - self.num_train_timesteps // self.num_inference_steps
        a_t, a_prev = self.alphas_cumprod[t], self._ac(prev_t)
        b_t = np.float32(1) - a_t
        x0 = (x - np.sqrt(b_t) * eps) / np.sqrt(a_t)
        return (np.sqrt(a_prev) * x0 + np.sqrt(np.float32(1) - a_prev) * eps).astype(np.float32)

    def next_step(self, eps, t, x):
        cur, nxt = min(t - self.num_train_timesteps // self.num_inference_steps, 999), t
        a_t, a_next = self._ac(cur), self.alphas_cumprod[nxt]
        b_t = np.float32(1) - a_t
        x0 = (x - np.sqrt(b_t) * eps) / np.sqrt(a_t)
        return (np.sqrt(a_next) * x0 + np.sqrt(np.float32(1) - a_next) * eps).astype(np.float32)


def cfg(noise_pred: np.ndarray, guidance_scale: float, fast: bool) -> np.ndarray:
    """pipeline_tuneavideo.py:409-415: u + g (t - u); fast mode keeps the source row unguided."""
    u, t = np.split(noise_pred, 2)
    out = (u + np.float32(guidance_scale) * (t - u)).astype(np.float32)
    if fast:
        out[0] = t[0]
    return out
