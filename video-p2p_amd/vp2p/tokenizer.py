"""Deterministic, offline stand-in for the CLIP tokenizer interface the P2P path uses.

The reference loads ``CLIPTokenizer.from_pretrained(...)`` (run_videop2p.py:101) and uses only
``encode``, ``decode([id])`` (ptp_utils.py:266, seq_aligner.py:110-111) and ``__call__`` with
``padding="max_length"`` (pipeline_tuneavideo.py:153-159, run_videop2p.py:541-552).  No CLIP
vocabulary exists offline, so this tokenizer reproduces the *shape* of CLIP tokenisation that the
P2P host logic depends on:

* BOS 49406 / EOS 49407 framing, EOS used as padding, ``model_max_length`` = 77;
* lower-casing;
* hyphenated words split into ``word``, ``-``, ``word`` pieces (CLIP BPE splits ``Spider-Man``
  into three tokens), so 1->k word replacements and multi-token words exercise the ratio
  mappers (seq_aligner.py:171-174) and multi-index ``get_word_inds`` results;
* ``decode([id])`` returns the piece text, so ``get_word_inds``'s length accumulation works.

Ids are a stable CRC32 hash of the piece (no global state), so every process assigns the same id.
Any tokenizer object with the same four methods (e.g. a real ``CLIPTokenizer``) can be passed to
the controllers instead.
"""
from __future__ import annotations

import re
import zlib
from typing import Dict, List, Sequence, Union

import torch

BOS_ID = 49406
EOS_ID = 49407
_ID_RANGE = 49000 - 1000


def _pieces(word: str) -> List[str]:
    out: List[str] = []
    for part in re.split(r"(-)", word.lower()):
        if part:
            out.append(part)
    return out


def piece_id(piece: str) -> int:
    return 1000 + zlib.crc32(piece.encode("utf-8")) % _ID_RANGE


class _Encoding:
    def __init__(self, input_ids: torch.Tensor, attention_mask: torch.Tensor):
        self.input_ids = input_ids
        self.attention_mask = attention_mask

    def __getitem__(self, key):
        return getattr(self, key)


class SyntheticCLIPTokenizer:
    model_max_length = 77
    bos_token_id = BOS_ID
    eos_token_id = EOS_ID
    pad_token_id = EOS_ID

    def __init__(self):
        self._rev: Dict[int, str] = {BOS_ID: "<|startoftext|>", EOS_ID: "<|endoftext|>"}

    def _ids(self, text: str) -> List[int]:
        ids = []
        for word in text.split():
            for p in _pieces(word):
                i = piece_id(p)
                prev = self._rev.get(i)
                if prev is not None and prev != p:
                    raise RuntimeError(f"synthetic tokenizer id collision: {prev!r} vs {p!r}")
                self._rev[i] = p
                ids.append(i)
        return ids

    def encode(self, text: str) -> List[int]:
        return [BOS_ID] + self._ids(text) + [EOS_ID]

    def decode(self, ids: Sequence[int]) -> str:
        return "".join(self._rev.get(int(i), "") for i in ids)

    def __call__(self, prompts: Union[str, List[str]], padding="max_length", max_length=None,
                 truncation=False, return_tensors="pt"):
        if isinstance(prompts, str):
            prompts = [prompts]
        rows = [self.encode(p) for p in prompts]
        if padding == "max_length":
            width = max_length or self.model_max_length
        else:  # "longest"
            width = max(len(r) for r in rows)
        ids = torch.full((len(rows), width), EOS_ID, dtype=torch.int64)
        mask = torch.zeros((len(rows), width), dtype=torch.int64)
        for i, r in enumerate(rows):
            if truncation and len(r) > width:
                r = r[: width - 1] + [EOS_ID]
            n = min(len(r), width)
            ids[i, :n] = torch.tensor(r[:n])
            mask[i, :n] = 1
        return _Encoding(ids, mask)
