"""CLIP byte-level BPE tokenizer, read from a local ``vocab.json`` + ``merges.txt``.

The reference loads ``CLIPTokenizer.from_pretrained(pretrained_model_path, subfolder="tokenizer")``
(run_videop2p.py:101, pipeline_tuneavideo.py:153-159) and the P2P host logic uses only
``encode``, ``decode([id])`` (ptp_utils.py:266, seq_aligner.py:110-111) and ``__call__`` with
``padding="max_length"``.  This module restates the published CLIP BPE algorithm (OpenAI CLIP
``simple_tokenizer.py``; the same algorithm as ``transformers.CLIPTokenizer``) so a real SD-1.5
tokenizer directory gives the reference's token ids without a network or ``transformers``:

1. text clean-up: whitespace collapse and lower-case, as ``transformers``' CLIP tokenizers do
   without ftfy (no HTML unescape, unlike OpenAI's ``simple_tokenizer``: ``&amp;`` stays three
   pieces);
2. pre-tokenisation with CLIP's regex (special tokens, contractions, letter runs, single digits,
   punctuation runs);
3. each piece is mapped byte -> printable unicode (GPT-2 ``bytes_to_unicode``), its last symbol
   gets the ``</w>`` end-of-word suffix, and merges are applied lowest-rank-first until none
   applies;
4. BOS/EOS framing; EOS pads to ``model_max_length`` (77).

``decode`` joins the token strings, maps back to bytes and turns ``</w>`` into a space, so
``decode([id]).strip()`` is the piece text ``get_word_inds`` accumulates (ptp_utils.py:266-272).
``load_tokenizer`` loads this tokenizer from a directory (raising if the files are missing) and
returns the offline synthetic one only when asked for explicitly.
"""
from __future__ import annotations

import json
import logging
import os
from functools import lru_cache
from typing import Dict, List, Optional, Sequence, Tuple, Union

import regex
import torch

from .tokenizer import SyntheticCLIPTokenizer, _Encoding

log = logging.getLogger("vp2p")

BOS = "<|startoftext|>"
EOS = "<|endoftext|>"
_PAT = regex.compile(
    r"""<\|startoftext\|>|<\|endoftext\|>|'s|'t|'re|'ve|'m|'ll|'d|[\p{L}]+|[\p{N}]|[^\s\p{L}\p{N}]+""",
    regex.IGNORECASE)


@lru_cache()
def bytes_to_unicode() -> Dict[int, str]:
    """GPT-2/CLIP reversible byte -> printable-unicode table (256 entries)."""
    keep = list(range(ord("!"), ord("~") + 1)) + list(range(ord("¡"), ord("¬") + 1)) + \
        list(range(ord("®"), ord("ÿ") + 1))
    table = {b: chr(b) for b in keep}
    extra = 0
    for b in range(256):
        if b not in table:
            table[b] = chr(256 + extra)
            extra += 1
    return table


def _clean(text: str) -> str:
    return regex.sub(r"\s+", " ", text).strip().lower()


def _pairs(word: Tuple[str, ...]):
    return {(word[i], word[i + 1]) for i in range(len(word) - 1)}


class CLIPBPETokenizer:
    model_max_length = 77

    def __init__(self, encoder: Dict[str, int], merges: Sequence[Tuple[str, str]]):
        self.encoder = dict(encoder)
        self.decoder = {v: k for k, v in self.encoder.items()}
        self.bpe_ranks = {tuple(m): i for i, m in enumerate(merges)}
        self.byte_encoder = bytes_to_unicode()
        self.byte_decoder = {v: k for k, v in self.byte_encoder.items()}
        for tok in (BOS, EOS):
            if tok not in self.encoder:
                raise ValueError(f"vocab has no {tok!r}")
        self.bos_token_id = self.encoder[BOS]
        self.eos_token_id = self.encoder[EOS]
        self.pad_token_id = self.eos_token_id
        self._cache: Dict[str, List[str]] = {BOS: [BOS], EOS: [EOS]}

    @classmethod
    def from_files(cls, vocab_file: str, merges_file: str) -> "CLIPBPETokenizer":
        with open(vocab_file, encoding="utf-8") as fh:
            encoder = json.load(fh)
        merges = []
        with open(merges_file, encoding="utf-8") as fh:
            for line in fh.read().split("\n"):
                if not line or line.startswith("#version"):
                    continue
                a, b = line.split()
                merges.append((a, b))
        return cls(encoder, merges)

    @classmethod
    def from_pretrained(cls, path: str, subfolder: Optional[str] = None) -> "CLIPBPETokenizer":
        d = os.path.join(path, subfolder) if subfolder else path
        return cls.from_files(os.path.join(d, "vocab.json"), os.path.join(d, "merges.txt"))

    def bpe(self, piece: str) -> List[str]:
        hit = self._cache.get(piece)
        if hit is not None:
            return hit
        word = tuple(piece[:-1]) + (piece[-1] + "</w>",)
        pairs = _pairs(word)
        while pairs:
            best = min(pairs, key=lambda p: self.bpe_ranks.get(p, float("inf")))
            if best not in self.bpe_ranks:
                break
            a, b = best
            out: List[str] = []
            i = 0
            while i < len(word):
                if i < len(word) - 1 and word[i] == a and word[i + 1] == b:
                    out.append(a + b)
                    i += 2
                else:
                    out.append(word[i])
                    i += 1
            word = tuple(out)
            if len(word) == 1:
                break
            pairs = _pairs(word)
        self._cache[piece] = list(word)
        return self._cache[piece]

    def tokenize(self, text: str) -> List[str]:
        toks: List[str] = []
        for piece in _PAT.findall(_clean(text)):
            if piece in (BOS, EOS):
                toks.append(piece)
                continue
            toks.extend(self.bpe("".join(self.byte_encoder[b] for b in piece.encode("utf-8"))))
        return toks

    def _ids(self, text: str) -> List[int]:
        unk = self.eos_token_id   # CLIP's unk token is <|endoftext|>
        return [self.encoder.get(t, unk) for t in self.tokenize(text)]

    def encode(self, text: str) -> List[int]:
        return [self.bos_token_id] + self._ids(text) + [self.eos_token_id]

    def decode(self, ids: Sequence[int]) -> str:
        # special-token and "</w>" characters are printable ASCII, which the byte table maps to
        # themselves, so one byte-decode covers every token
        text = "".join(self.decoder.get(int(i), "") for i in ids)
        raw = bytearray(self.byte_decoder[c] for c in text)
        return raw.decode("utf-8", errors="replace").replace("</w>", " ").strip()

    def __call__(self, prompts: Union[str, List[str]], padding="max_length", max_length=None,
                 truncation=False, return_tensors="pt"):
        if isinstance(prompts, str):
            prompts = [prompts]
        rows = [self.encode(p) for p in prompts]
        width = (max_length or self.model_max_length) if padding == "max_length" else max(map(len, rows))
        ids = torch.full((len(rows), width), self.pad_token_id, dtype=torch.int64)
        mask = torch.zeros((len(rows), width), dtype=torch.int64)
        for i, r in enumerate(rows):
            if truncation and len(r) > width:
                r = r[: width - 1] + [self.eos_token_id]
            n = min(len(r), width)
            ids[i, :n] = torch.tensor(r[:n])
            mask[i, :n] = 1
        return _Encoding(ids, mask)


def load_tokenizer(path: Optional[str] = None, subfolder: Optional[str] = "tokenizer", synthetic: bool = False):
    """The real CLIP BPE from ``<path>/<subfolder>/{vocab.json,merges.txt}`` (run_videop2p.py:101).

    The offline synthetic tokenizer is returned only when asked for explicitly (``path=None`` or
    ``synthetic=True``): a path whose vocabulary files are missing raises ``FileNotFoundError``
    instead of silently tokenising with made-up ids (which would give every mapper, word index
    and LocalBlend layer a tokenisation different from CLIP's)."""
    if synthetic or not path:
        log.info("vp2p: using the synthetic CLIP tokenizer (no vocabulary files)")
        return SyntheticCLIPTokenizer()
    tried = []
    for d in ((os.path.join(path, subfolder) if subfolder else path), path):
        tried.append(d)
        if os.path.isfile(os.path.join(d, "vocab.json")) and os.path.isfile(os.path.join(d, "merges.txt")):
            log.info("vp2p: CLIP BPE tokenizer from %s", d)
            return CLIPBPETokenizer.from_pretrained(d)
    raise FileNotFoundError(f"no CLIP vocab.json + merges.txt under {tried}; pass synthetic=True for the offline "
                            "synthetic tokenizer")
