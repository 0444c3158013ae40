"""Training / validation driver with the reference trainer's semantics (``Manager``, src/main.py:36-251).

Per step (src/main.py:137-169): batch to HBM, forward, ``zero_grad``, ``backward``, optimizer step,
scheduler step; the reported metrics are the mean total loss, PPL = exp(mean LM loss) and emotion
accuracy.  The reference syncs the host three times per step (``loss.item()`` and a duplicate
full-vocabulary CE over the logits to get the LM loss); here the fused step already returns the LM
loss (``loss_lm``, the same masked mean), and all metrics accumulate on the device and are read once
per epoch.  Validation (src/main.py:206-251) runs the inference forward under ``no_grad``.

Checkpoints use the reference's keys (src/main.py:184-196: ``model_state_dict``, ``optim_state_dict``,
``sched_state_dict``, ``ppl``, ``epoch``) and file name pattern; the model's state_dict keys are the
reference's and the optimizer state is written in the reference's per-tensor AdamW format
(``FusedAdamW.reference_state_dict``), so checkpoints interchange with the reference in both
directions (``load`` accepts either optimizer format).  They are written with ``torch.save`` and read
back with ``torch.load(weights_only=True)``.

Data parallel: pass a ``process_group``; each rank iterates its own shard (e.g. a
``DistributedSampler``; every rank must run the same number of steps), the per-step losses are
already global means (the loss normalisers are all-reduced before each forward), so the epoch loss
is their rank sum averaged over one rank's steps; correct predictions and samples are summed.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass
from typing import Dict, Iterable, Optional, Tuple

import torch

from .dataset import DevicePrefetcher


@dataclass
class EpochStats:
    loss: float
    ppl: float
    acc: float        # percent
    steps: int
    samples: int


class Trainer:
    def __init__(self, model, optim, sched=None, device: Optional[torch.device] = None, process_group=None,
                 ckpt_dir: Optional[str] = None):
        self.model, self.optim, self.sched = model, optim, sched
        self.device = device if device is not None else model.flat.device
        self.pg = process_group
        self.ckpt_dir = ckpt_dir
        self.best_ppl = float("inf")
        self.last_epoch = 0
        # called after every training step (after the optimizer and scheduler steps): diagnostics / tests
        self.step_hook = None

    # ---- one pass -------------------------------------------------------------------------
    def _pass(self, loader: Iterable[Dict[str, torch.Tensor]], train: bool) -> EpochStats:
        dev = self.device
        acc = torch.zeros(3, dtype=torch.float64, device=dev)   # Σ loss, Σ lm loss, Σ correct
        steps = samples = 0
        for batch in DevicePrefetcher(loader, dev):
            kw = dict(input_ids=batch["input_ids"], token_type_ids=batch["token_type_ids"], labels=batch["labels"],
                      emotion_labels=batch["emotion_labels"], caption_ids=batch["caption_ids"],
                      imgs=batch.get("visual_feat"), auds=batch.get("audio_feat"))
            if train:
                out = self.model(**kw)
                self.optim.zero_grad()
                out.loss.backward()
                self.optim.step()
                if self.sched is not None:
                    self.sched.step()
                if self.step_hook is not None:
                    self.step_hook()
            else:
                with torch.no_grad():
                    out = self.model(**kw)
            acc[0] += out.loss.detach().double()
            acc[1] += out.loss_lm.detach().double()
            acc[2] += (out.emotion_logits.argmax(-1) == kw["emotion_labels"]).sum().double()
            steps += 1
            samples += kw["input_ids"].shape[0]
        tot = torch.tensor([steps, samples], dtype=torch.float64, device=dev)
        world = 1
        if self.pg is not None:
            import torch.distributed as dist
            world = dist.get_world_size(self.pg)
            dist.all_reduce(acc, group=self.pg)
            dist.all_reduce(tot, group=self.pg)
        a, t = acc.tolist(), tot.tolist()
        # Under DP each rank's loss is its share of the global step mean (local sums over the global
        # label counts), so the rank sum is the global mean of one step: divide by the steps one rank
        # ran (every rank runs the same number), not by the steps summed over ranks.
        n_steps = max(t[0] / world, 1.0)
        lm = a[1] / n_steps
        ppl = math.exp(lm) if lm < 700 else float("inf")
        if math.isnan(ppl):
            ppl = 1e8  # src/main.py:248-249
        return EpochStats(loss=a[0] / n_steps, ppl=ppl, acc=100.0 * a[2] / max(t[1], 1.0), steps=int(n_steps),
                          samples=int(t[1]))

    def train_epoch(self, loader) -> EpochStats:
        self.model.train()
        return self._pass(loader, True)

    def validation(self, loader) -> EpochStats:
        self.model.eval()
        return self._pass(loader, False)

    def train(self, train_loader, valid_loader, num_epochs: int, log=print,
              seed: Optional[int] = None) -> Tuple[EpochStats, EpochStats]:
        """src/main.py:125-204: epochs of training + validation, keeping the best-PPL checkpoint.  ``seed``: as the
        reference's ``fix_seed(args.seed)`` at the start of ``train()`` (src/main.py:124,284-289) — seeds torch,
        numpy and ``random``, and re-derives the model's dropout mask stream from it, so two runs from the same
        weights give identical epoch metrics."""
        if seed is not None:
            import random
            import numpy as np
            random.seed(seed)
            np.random.seed(seed)
            torch.manual_seed(seed)
            if hasattr(self.model, "reseed_dropout"):
                self.model.reseed_dropout()
        tr = va = None
        start = self.last_epoch + 1
        for epoch in range(start, start + num_epochs):
            tr = self.train_epoch(train_loader)
            log(f"Epoch {epoch}: Train Loss: {tr.loss:.4f} | Train PPL: {tr.ppl:.4f} | "
                f"Train Emotion Acc: {tr.acc:.2f}%")
            self.last_epoch += 1
            va = self.validation(valid_loader)
            if va.ppl < self.best_ppl:
                self.best_ppl = va.ppl
                if self.ckpt_dir is not None and hasattr(self.model, "consolidate_"):
                    self.model.consolidate_()  # collective: every rank (the sharded optimizer update)
                if self.ckpt_dir is not None and self._rank0():
                    path = os.path.join(self.ckpt_dir, f"best_ckpt_epoch={epoch}_valid_ppl={self.best_ppl:.4f}.ckpt")
                    self.save(path)
                    log(f"Current best checkpoint is saved: {path}")
            log(f"Best valid PPL: {self.best_ppl:.4f} | valid loss {va.loss:.4f} | valid PPL {va.ppl:.4f} | "
                f"valid Emotion Acc: {va.acc:.2f}%")
        return tr, va

    # ---- checkpoints ----------------------------------------------------------------------
    def _rank0(self) -> bool:
        if self.pg is None:
            return True
        import torch.distributed as dist
        return dist.get_rank(self.pg) == 0

    def state_dict(self) -> Dict:
        # the optimizer part in the reference's per-tensor AdamW format when the optimizer can write it, so the
        # reference's resume (src/main.py:107) loads this checkpoint and vice versa
        ref_fmt = getattr(self.optim, "reference_state_dict", None)
        optim_sd = ref_fmt() if ref_fmt is not None and getattr(self.optim, "model", None) is not None \
            else self.optim.state_dict()
        return {"model_state_dict": {k: v.detach().clone() for k, v in self.model.state_dict().items()},
                "optim_state_dict": optim_sd,
                "sched_state_dict": self.sched.state_dict() if self.sched is not None else None,
                "ppl": self.best_ppl, "epoch": self.last_epoch}

    def save(self, path: str) -> None:
        os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
        torch.save(self.state_dict(), path)

    def load(self, path: str, resume: bool = True) -> None:
        """src/main.py:98-119: model weights (strict=False, as the reference), and for a resumed
        training run the optimizer / scheduler state, best PPL and epoch."""
        ck = torch.load(path, map_location=self.device, weights_only=True)
        self.model.load_state_dict(ck["model_state_dict"], strict=False)
        if resume:
            self.optim.load_state_dict(ck["optim_state_dict"])
            if self.sched is not None and ck.get("sched_state_dict") is not None:
                self.sched.load_state_dict(ck["sched_state_dict"])
            self.best_ppl = ck.get("ppl", float("inf"))
            self.last_epoch = ck["epoch"]
