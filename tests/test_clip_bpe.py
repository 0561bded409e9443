"""CLIP BPE tokenizer (vp2p.clip_bpe) against transformers.CLIPTokenizer on a small synthetic
vocab/merges pair written to a temp dir (no CLIP vocabulary ships offline), plus the P2P host
logic (get_word_inds / mappers / equalizer, ptp_utils.py:258-310, seq_aligner.py) run through
both tokenizers.  CPU only."""
import json

import numpy as np
import pytest
import torch

from vp2p import prompt_align as PA
from vp2p.clip_bpe import CLIPBPETokenizer, bytes_to_unicode, load_tokenizer
from vp2p.tokenizer import SyntheticCLIPTokenizer

# fully merged words become one token; the partial ones stay multi-token (CLIP splits rare words)
FULL = ["a", "rabbit", "is", "jumping", "on", "the", "grass", "man", "car", "penguin", "running",
        "in", "snow", "driving", "road", "-", "spider", "'s", "kitten"]
PARTIAL = {"origami": 4, "lego": 2, "watercolor": 6}
PROMPTS = [
    "a rabbit is jumping on the grass",
    "a origami rabbit is jumping on the grass",
    "a lego rabbit is  jumping on the grass",
    "a spider-man is driving a car on the road",
    "a penguin is running in the snow, watercolor",
    "The Kitten's  car 42 &amp; more!",
]


def _write_vocab(tmp_path):
    bu = list(bytes_to_unicode().values())
    vocab = bu + [c + "</w>" for c in bu]
    merges = []

    def add(word, n_merge=None):
        enc = "".join(bytes_to_unicode()[b] for b in word.encode())
        syms = list(enc[:-1]) + [enc[-1] + "</w>"]
        steps = len(syms) - 1 if n_merge is None else n_merge
        cur = syms[0]
        for s in syms[1:steps + 1]:
            m = (cur, s)
            if m not in merges:
                merges.append(m)
                if cur + s not in vocab:
                    vocab.append(cur + s)
            cur = cur + s

    for w in FULL:
        add(w)
    for w, n in PARTIAL.items():
        add(w, n)
    vocab += ["<|startoftext|>", "<|endoftext|>"]
    enc = {t: i for i, t in enumerate(dict.fromkeys(vocab))}
    (tmp_path / "vocab.json").write_text(json.dumps(enc), encoding="utf-8")
    (tmp_path / "merges.txt").write_text(
        "#version: 0.2\n" + "\n".join(f"{a} {b}" for a, b in merges) + "\n", encoding="utf-8")
    return tmp_path


@pytest.fixture(scope="module")
def toks(tmp_path_factory):
    d = _write_vocab(tmp_path_factory.mktemp("clip_tok"))
    transformers = pytest.importorskip("transformers")
    hf = transformers.CLIPTokenizer(str(d / "vocab.json"), str(d / "merges.txt"))
    return CLIPBPETokenizer.from_pretrained(str(d)), hf, d


def test_encode_matches_transformers(toks):
    ours, hf, _ = toks
    for p in PROMPTS:
        assert ours.encode(p) == hf.encode(p), p


def test_decode_single_ids_match_transformers(toks):
    ours, hf, _ = toks
    for p in PROMPTS:
        for i in hf.encode(p):
            assert ours.decode([i]) == hf.decode([i]), (p, i)
    assert ours.decode(ours.encode(PROMPTS[0])[1:-1]) == PROMPTS[0]


def test_call_padding_matches_transformers(toks):
    ours, hf, _ = toks
    a = ours(PROMPTS, padding="max_length", max_length=77, truncation=True, return_tensors="pt")
    b = hf(PROMPTS, padding="max_length", max_length=77, truncation=True, return_tensors="pt")
    assert torch.equal(a.input_ids, b.input_ids)
    long = " ".join(["rabbit"] * 100)
    assert torch.equal(ours([long], max_length=77, truncation=True).input_ids,
                       hf([long], padding="max_length", max_length=77, truncation=True,
                          return_tensors="pt").input_ids)


def test_multi_token_words_and_host_logic_agree(toks):
    ours, hf, _ = toks
    assert len(ours.encode("origami")) > 3     # partial merges: one word, several tokens
    for p in PROMPTS[:4]:
        for w in ("rabbit", "origami", "lego", "car", "man", 1, 3):
            np.testing.assert_array_equal(PA.get_word_inds(p, w, ours), PA.get_word_inds(p, w, hf))
    np.testing.assert_array_equal(PA.get_word_inds(PROMPTS[1], "origami", ours),
                                  np.arange(2, 2 + len(ours.encode("origami")) - 2))
    for pair in (PROMPTS[:2], [PROMPTS[0], PROMPTS[2]]):
        m1, a1 = PA.get_refinement_mapper(pair, ours)
        m2, a2 = PA.get_refinement_mapper(pair, hf)
        assert torch.equal(m1, m2) and torch.equal(a1, a2)
    r1 = PA.get_replacement_mapper([PROMPTS[0], "a lego is jumping on the grass"], ours)
    r2 = PA.get_replacement_mapper([PROMPTS[0], "a lego is jumping on the grass"], hf)
    assert torch.equal(r1, r2)
    e1 = PA.get_equalizer(PROMPTS[1], ("origami",), (2.0,), ours)
    e2 = PA.get_equalizer(PROMPTS[1], ("origami",), (2.0,), hf)
    assert torch.equal(e1, e2)


def test_load_tokenizer_picks_files(toks, tmp_path):
    _, _, d = toks
    assert isinstance(load_tokenizer(str(d), subfolder=None), CLIPBPETokenizer)
    with pytest.raises(FileNotFoundError):        # a path without the files is an error, not a fallback
        load_tokenizer(str(tmp_path))
    assert isinstance(load_tokenizer(None), SyntheticCLIPTokenizer)
    assert isinstance(load_tokenizer(str(tmp_path), synthetic=True), SyntheticCLIPTokenizer)
