"""Synthetic MELD / IEMOCAP-shaped batches with the reference's batch contract.

The batch layout follows ``CustomDataset`` / ``PadCollate`` (src/custom_dataset.py:9-132):

* ``input_ids``      [B, S] int64 — concatenated dialogue turns (:49)
* ``token_type_ids`` [B, S] int64 — sp1 for even turns, sp2 for odd turns (:54-56)
* ``labels``         [B, S] int64 — ``-100`` on the context, LM targets right-aligned on the last
                     turn ending in eos (:59-68)
* ``emotion_labels`` [B]    int64 — one of 7 emotions (:75)
* ``caption_ids``    [B, S] int64 — keyframe caption tokens; the reference forces caption length = S
                     (src/model.py:461)
* ``visual_feat``    [B, Tv, E] f32 — BLIP vision features, row 0 used (``imgs[i][0]`` src/model.py:497)
* ``audio_feat``     [B, E] f32 — mean-pooled wav2vec2 vector (``auds[i]`` src/model.py:498)

Shapes per SURVEY §8(d): MELD-shape S=128 in 5 turns, IEMOCAP-shape S=512 in 20 turns.
Real MELD/IEMOCAP pickles are not available offline; the data is synthetic (stated in bench output).
"""
from __future__ import annotations

from typing import Dict

import torch

from .config import EOS_ID, GPT2_BASE_VOCAB, NUM_EMOTIONS, SP1_ID, SP2_ID


def turn_lengths(S: int, n_turns: int, g: torch.Generator, min_len: int = 8) -> list:
    """Split S tokens into n_turns turns, each >= min_len, by a seeded multinomial."""
    if n_turns * min_len > S:
        min_len = max(1, S // n_turns)
    rest = S - n_turns * min_len
    extra = torch.multinomial(torch.ones(n_turns), rest, replacement=True, generator=g) if rest > 0 else \
        torch.zeros(0, dtype=torch.long)
    lens = torch.full((n_turns,), min_len, dtype=torch.long)
    lens += torch.bincount(extra, minlength=n_turns)
    return lens.tolist()


def synthetic_batch(B: int, S: int, n_turns: int = 5, feat_dim: int = 768, seed: int = 0,
                    vocab_lo: int = 0, vocab_hi: int = GPT2_BASE_VOCAB, visual_rows: int = 1,
                    with_features: bool = True, sp1: int = SP1_ID, sp2: int = SP2_ID,
                    eos: int = EOS_ID) -> Dict[str, torch.Tensor]:
    g = torch.Generator().manual_seed(seed)
    input_ids = torch.randint(vocab_lo, vocab_hi, (B, S), generator=g)
    token_type_ids = torch.empty(B, S, dtype=torch.long)
    labels = torch.full((B, S), -100, dtype=torch.long)
    for b in range(B):
        lens = turn_lengths(S, n_turns, g)
        o = 0
        for c, ln in enumerate(lens):
            token_type_ids[b, o:o + ln] = sp1 if c % 2 == 0 else sp2      # custom_dataset.py:55
            o += ln
        last = lens[-1]
        labels[b, S - last:] = input_ids[b, S - last:]                   # right-aligned target :62-64
        labels[b, S - 1] = eos                                           # + [eos] :60
    emotion_labels = torch.randint(0, NUM_EMOTIONS, (B,), generator=g)
    caption_ids = torch.randint(vocab_lo, vocab_hi, (B, S), generator=g)
    out = dict(input_ids=input_ids, token_type_ids=token_type_ids, labels=labels,
               emotion_labels=emotion_labels, caption_ids=caption_ids)
    if with_features:
        out["visual_feat"] = 0.1 * torch.randn(B, visual_rows, feat_dim, generator=g)
        out["audio_feat"] = 0.1 * torch.randn(B, feat_dim, generator=g)
    return out


MELD_SHAPE = dict(S=128, n_turns=5)
IEMOCAP_SHAPE = dict(S=512, n_turns=20)
