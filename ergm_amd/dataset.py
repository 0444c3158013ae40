"""Real-data input pipeline: the reference's sample construction and padding collate, plus an
asynchronous host→HBM prefetcher.

``DialogueDataset`` restates ``CustomDataset`` (src/custom_dataset.py:9-101) over the same
in-memory schema the reference unpickles —

* main data:    ``{"txt": [dialogue][utterance] -> list of turn token lists, "img": [dialogue][0] -> E-vector,
                  "aud": [dialogue][0] -> E-vector, "label": [dialogue][utterance] -> LM target token list}``
* context data: ``{"context": [dialogue][utterance] -> caption token list, "label": [dialogue][utterance] -> emotion id}``

Per utterance (src/custom_dataset.py:44-81): input ids = the concatenated turns (skipped when
>= 1024 tokens); token types = sp1 for even turns, sp2 for odd; LM labels = target[2:-2] + [eos],
right-aligned with -100 on the left, or the input padded with eos when the target is longer; the
dialogue's first visual / audio vectors; the context tokens; the emotion label.

``PadCollate`` restates the reference collate (src/custom_dataset.py:103-132): pad ids and token
types with eos, labels with -100, to the longest sequence in the batch (optionally rounded up to a
multiple, which bounds the number of distinct shapes the executor plans for).  It returns the
build's keyword batch: ``visual_feat`` [B, E] (the reference model reads ``imgs[i][0]``,
src/model.py:497), ``audio_feat`` [B, E], and ``caption_ids`` [B, S] — the context tokens cut or
eos-padded to S, since the reference forces caption length == text length (src/model.py:461) and
its trainer never wires captions; this wiring is the build's.

Padding needs no kernel support: the reference trains without an attention mask, so padded
positions attend and are attended exactly as in the reference; their labels are -100.

Loading the pickles themselves is the caller's business (they are the user's own files); the
reference's data is not shipped and nothing here unpickles.
"""
from __future__ import annotations

from itertools import chain
from typing import Dict, List, Optional, Sequence

import torch

from .config import EOS_ID, SP1_ID, SP2_ID


class DialogueDataset(torch.utils.data.Dataset):
    def __init__(self, data: Dict, context_label: Dict, sp1_id: int = SP1_ID, sp2_id: int = SP2_ID,
                 eos_id: int = EOS_ID, max_len: int = 1024):
        texts, videos, audios, targets = data["txt"], data["img"], data["aud"], data["label"]
        contexts, emotions = context_label["context"], context_label["label"]
        self.samples: List[tuple] = []
        for i in range(len(texts)):
            if not (len(texts[i]) == len(targets[i]) == len(contexts[i]) == len(emotions[i])):
                raise ValueError(f"dialogue {i}: texts / targets / contexts / emotion labels differ in length")
            vis = torch.as_tensor(videos[i][0], dtype=torch.float32).reshape(-1)
            aud = torch.as_tensor(audios[i][0], dtype=torch.float32).reshape(-1)
            for j, turns in enumerate(texts[i]):
                ids = list(chain.from_iterable(turns))
                if len(ids) >= max_len:
                    continue
                tt = list(chain.from_iterable([sp1_id if c % 2 == 0 else sp2_id] * len(t) for c, t in enumerate(turns)))
                lm = list(targets[i][j][2:-2]) + [eos_id]
                gap = len(ids) - len(lm)
                if gap > 0:
                    lm = [-100] * gap + lm
                elif gap < 0:
                    ids = ids + [eos_id] * (-gap)
                    tt = tt + [tt[-1]] * (-gap)
                self.samples.append((ids, tt, lm, vis, aud, list(contexts[i][j]), int(emotions[i][j])))

    def __len__(self) -> int:
        return len(self.samples)

    def __getitem__(self, k: int) -> tuple:
        return self.samples[k]


class PadCollate:
    def __init__(self, eos_id: int = EOS_ID, pad_multiple: int = 1):
        self.eos_id = eos_id
        self.pad_multiple = max(1, pad_multiple)

    def __call__(self, batch: Sequence[tuple]) -> Dict[str, torch.Tensor]:
        S = max(len(b[0]) for b in batch)
        S = -(-S // self.pad_multiple) * self.pad_multiple
        B = len(batch)
        ids = torch.full((B, S), self.eos_id, dtype=torch.long)
        tt = torch.full((B, S), self.eos_id, dtype=torch.long)
        labels = torch.full((B, S), -100, dtype=torch.long)
        cap = torch.full((B, S), self.eos_id, dtype=torch.long)
        for r, (i, t, lm, _, _, ctx, _) in enumerate(batch):
            n = len(i)
            ids[r, :n] = torch.as_tensor(i)
            tt[r, :n] = torch.as_tensor(t)
            labels[r, :n] = torch.as_tensor(lm)
            c = ctx[:S]
            if c:
                cap[r, :len(c)] = torch.as_tensor(c)
        return {"input_ids": ids, "token_type_ids": tt, "labels": labels,
                "visual_feat": torch.stack([b[3] for b in batch]), "audio_feat": torch.stack([b[4] for b in batch]),
                "caption_ids": cap, "emotion_labels": torch.as_tensor([b[6] for b in batch], dtype=torch.long)}


class DevicePrefetcher:
    """Iterates a loader of keyword batches, staging batch k+1 into HBM (pinned host memory,
    non-blocking copies on a dedicated stream) while step k computes; the consumer stream waits on
    the copy's event, never the host."""

    def __init__(self, loader, device: torch.device):
        self.loader, self.device = loader, device
        self.stream = torch.cuda.Stream(device) if device.type == "cuda" else None

    def _stage(self, batch: Dict[str, torch.Tensor]):
        if self.stream is None:
            return {k: v.to(self.device) for k, v in batch.items()}, None
        with torch.cuda.stream(self.stream):
            out = {k: (v if v.is_pinned() else v.pin_memory()).to(self.device, non_blocking=True)
                   for k, v in batch.items()}
            ev = torch.cuda.Event()
            ev.record(self.stream)
        return out, ev

    def __iter__(self):
        it = iter(self.loader)
        nxt: Optional[tuple] = None
        try:
            nxt = self._stage(next(it))
        except StopIteration:
            return
        while nxt is not None:
            cur, ev = nxt
            try:
                nxt = self._stage(next(it))
            except StopIteration:
                nxt = None
            if ev is not None:
                cs = torch.cuda.current_stream(self.device)
                cs.wait_event(ev)
                for v in cur.values():  # the copy stream's allocations are used on the compute stream
                    v.record_stream(cs)
            yield cur

    def __len__(self):
        return len(self.loader)
