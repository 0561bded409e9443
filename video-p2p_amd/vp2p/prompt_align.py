"""Prompt bookkeeping for P2P edits: word->token indices, token alignment mappers, per-step word
alphas and reweighting vectors.  Host-only, run once per controller.

Mirrors the reference functions (same names, arguments, results and errors):
  get_word_inds                    ptp_utils.py:258-276 (duplicate at seq_aligner.py:133-151)
  update_alpha_time_word           ptp_utils.py:279-289
  get_time_words_attention_alpha   ptp_utils.py:292-310
  get_refinement_mapper            seq_aligner.py:109-130 (Needleman-Wunsch, gap 0/match 1/mismatch -1)
  get_replacement_mapper           seq_aligner.py:154-197
  get_equalizer                    run_videop2p.py:372-381
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Tuple, Union

import numpy as np
import torch

MAX_NUM_WORDS = 77


def get_word_inds(text: str, word_place: Union[str, int], tokenizer) -> np.ndarray:
    words = text.split(" ")
    if isinstance(word_place, str):
        wanted = {i for i, w in enumerate(words) if w == word_place}
    elif isinstance(word_place, int):
        wanted = {word_place}
    else:
        wanted = set(word_place)
    if not wanted:
        return np.array([])
    # decoded token pieces (BOS/EOS dropped); a word ends once its characters are consumed
    pieces = [tokenizer.decode([t]).strip("#") for t in tokenizer.encode(text)][1:-1]
    out, word, used = [], 0, 0
    for tok, piece in enumerate(pieces, start=1):
        used += len(piece)
        if word in wanted:
            out.append(tok)
        if used >= len(words[word]):
            word, used = word + 1, 0
    return np.array(out)


def update_alpha_time_word(alpha: torch.Tensor, bounds: Union[float, Tuple[float, float]],
                           prompt_ind: int, word_inds=None) -> torch.Tensor:
    lo_f, hi_f = (0.0, bounds) if isinstance(bounds, float) else bounds
    n = alpha.shape[0]
    lo, hi = int(lo_f * n), int(hi_f * n)
    cols = torch.arange(alpha.shape[2]) if word_inds is None else torch.as_tensor(word_inds)
    window = torch.zeros(n, dtype=alpha.dtype)
    window[lo:hi] = 1
    alpha[:, prompt_ind, cols] = window[:, None].expand(n, len(cols)).to(alpha.dtype)
    return alpha


def get_time_words_attention_alpha(prompts: Sequence[str], num_steps: int,
                                   cross_replace_steps: Union[float, Dict[str, Tuple[float, float]]],
                                   tokenizer, max_num_words: int = MAX_NUM_WORDS) -> torch.Tensor:
    """(num_steps + 1, P - 1, 1, 1, 77) 0/1 word alphas: the default window for every word, then
    per-word windows for named words of the edited prompts."""
    steps = dict(cross_replace_steps) if isinstance(cross_replace_steps, dict) else {"default_": cross_replace_steps}
    steps.setdefault("default_", (0.0, 1.0))
    alpha = torch.zeros(num_steps + 1, len(prompts) - 1, max_num_words)
    for p in range(len(prompts) - 1):
        alpha = update_alpha_time_word(alpha, steps["default_"], p)
    for word, bounds in steps.items():
        if word == "default_":
            continue
        for p, prompt in enumerate(prompts[1:]):
            inds = get_word_inds(prompt, word, tokenizer)
            if len(inds):
                alpha = update_alpha_time_word(alpha, bounds, p, inds)
    return alpha.reshape(num_steps + 1, len(prompts) - 1, 1, 1, max_num_words)


# ------------------------------------------------------------------------------------------------
def _align(x: Sequence[int], y: Sequence[int]) -> List[Tuple[int, int]]:
    """Global alignment of token ids; returns (y index, x index or -1) for every y position that the
    traceback visits, in y order.  Ties prefer left (gap in x), then up, then diagonal."""
    n, m = len(x), len(y)
    score = np.zeros((n + 1, m + 1), np.int32)
    move = np.zeros((n + 1, m + 1), np.int8)   # 1 left, 2 up, 3 diag, 4 origin
    move[0, 1:], move[1:, 0], move[0, 0] = 1, 2, 4
    for i in range(1, n + 1):
        xi = x[i - 1]
        for j in range(1, m + 1):
            left, up = score[i, j - 1], score[i - 1, j]
            diag = score[i - 1, j - 1] + (1 if xi == y[j - 1] else -1)
            best = max(left, up, diag)
            score[i, j] = best
            move[i, j] = 1 if best == left else 2 if best == up else 3
    pairs = []
    i, j = n, m
    while (i > 0 or j > 0) and move[i, j] != 4:
        mv = move[i, j]
        if mv == 3:
            i, j = i - 1, j - 1
            pairs.append((j, i))
        elif mv == 1:
            j -= 1
            pairs.append((j, -1))
        else:
            i -= 1
    return pairs[::-1]


def get_mapper(x: str, y: str, tokenizer, max_len: int = MAX_NUM_WORDS):
    xs, ys = tokenizer.encode(x), tokenizer.encode(y)
    pairs = _align(xs, ys)
    k = len(pairs)
    src = torch.tensor([p[1] for p in pairs], dtype=torch.int64)
    alphas = torch.ones(max_len)
    alphas[:k] = (src != -1).float()
    mapper = torch.zeros(max_len, dtype=torch.int64)
    mapper[:k] = src
    mapper[k:] = len(ys) + torch.arange(max_len - len(ys))
    return mapper, alphas


def get_refinement_mapper(prompts: Sequence[str], tokenizer, max_len: int = MAX_NUM_WORDS):
    out = [get_mapper(prompts[0], p, tokenizer, max_len) for p in prompts[1:]]
    return torch.stack([m for m, _ in out]), torch.stack([a for _, a in out])


def get_replacement_mapper_(x: str, y: str, tokenizer, max_len: int = MAX_NUM_WORDS) -> torch.Tensor:
    wx, wy = x.split(" "), y.split(" ")
    if len(wx) != len(wy):
        raise ValueError(f"attention replacement edit can only be applied on prompts with the same"
                         f" length but prompt A has {len(wx)} words and prompt B has {len(wy)} words.")
    swapped = [i for i in range(len(wy)) if wy[i] != wx[i]]
    src = [get_word_inds(x, i, tokenizer) for i in swapped]
    dst = [get_word_inds(y, i, tokenizer) for i in swapped]
    mapper = np.zeros((max_len, max_len))
    i = j = c = 0
    while i < max_len and j < max_len:
        if c < len(src) and src[c][0] == i:
            s, d = src[c], dst[c]
            if len(s) == len(d):
                mapper[s, d] = 1
            else:
                mapper[np.ix_(s, d)] = 1 / len(d)
            c += 1
            i += len(s)
            j += len(d)
        else:
            # before the last swapped word the unchanged tokens map (i, j); after it the reference
            # writes the diagonal (j, j) (seq_aligner.py:178-185)
            mapper[(i if c < len(src) else j), j] = 1
            i += 1
            j += 1
    return torch.from_numpy(mapper).float()


def get_replacement_mapper(prompts: Sequence[str], tokenizer, max_len: int = MAX_NUM_WORDS) -> torch.Tensor:
    return torch.stack([get_replacement_mapper_(prompts[0], p, tokenizer, max_len) for p in prompts[1:]])


def get_equalizer(text: str, word_select, values, tokenizer) -> torch.Tensor:
    if isinstance(word_select, (int, str)):
        word_select = (word_select,)
    eq = torch.ones(1, MAX_NUM_WORDS)
    for word, val in zip(word_select, values):
        eq[:, get_word_inds(text, word, tokenizer)] = val
    return eq
