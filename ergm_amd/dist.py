"""Data-parallel synchronisation for the fused training step (one process per GPU).

The reference trains on one device (src/main.py:40-43) and has no collective; the build adds pure
data parallelism:

1. Loss normalisation.  The reference LM loss is a mean over the valid (!= -100) shifted labels of the
   whole batch and the emotion loss a mean over the batch (src/model.py:704-713).  Each rank therefore
   divides its local sums by the GLOBAL valid-label count (all-reduced before the forward) and by the
   global batch, so the SUM over ranks of local gradients equals the gradient of the concatenated
   global batch on one device.
2. Gradient all-reduce (SUM) of contiguous buckets of the flat gradient buffer, launched on a side
   stream as soon as the backward stage that finalises each bucket has been enqueued, so RCCL over
   xGMI overlaps the remaining backward.  The last bucket (caption K/V + wpe + wte) is final only after
   the embedding backward and cannot overlap.

Works with any torch.distributed backend: "nccl" (= RCCL on ROCm) on GPUs, "gloo" for CPU tests.
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import torch


class DPSync:
    def __init__(self, process_group=None, buckets: Optional[List[Tuple[int, int]]] = None):
        self.pg = process_group
        self.buckets = buckets or []
        self._works: List = []
        self._stream = None
        self._events: List = []

    @property
    def world(self) -> int:
        if self.pg is None:
            return 1
        import torch.distributed as dist
        return dist.get_world_size(self.pg)

    @property
    def rank(self) -> int:
        if self.pg is None:
            return 0
        import torch.distributed as dist
        return dist.get_rank(self.pg)

    @property
    def active(self) -> bool:
        return self.world > 1

    def reduce_count(self, counts: torch.Tensor) -> None:
        """In place: local valid-label counts (LM, emotion) -> global counts (before the forward).
        The loss means divide by these, so ranks with different batch sizes or ignored labels still
        sum to the single-process gradient of the concatenated batch."""
        if self.active:
            import torch.distributed as dist
            dist.all_reduce(counts, group=self.pg)

    def begin(self) -> None:
        self._works = []

    def _side(self, dev):
        if self._stream is None:
            self._stream = torch.cuda.Stream(dev)
        return self._stream

    def enqueue(self, grad: torch.Tensor, fn, key: int, wait=None) -> None:
        """Run ``fn()`` on the side stream once everything issued so far on the current stream is
        done (``key`` selects the reusable ordering event; fn launches work, it does not wait).
        ``wait(stream_handle)``, if given, adds a further dependency of the side stream (the executor's
        weight-gradient stream mark of the bucket, ergm_model_stage_wait)."""
        if not grad.is_cuda:
            fn()
            return
        cur = torch.cuda.current_stream(grad.device)
        side = self._side(grad.device)
        while len(self._events) <= key:
            from ._lib import HipEvent
            self._events.append(HipEvent(sync=True))
        ev = self._events[key]  # reused every step: the wait below is enqueued right after the record
        ev.record(cur.cuda_stream)
        ev.wait(side.cuda_stream)
        if wait is not None:
            wait(side.cuda_stream)
        with torch.cuda.stream(side):
            fn()

    def bucket_ready(self, k: int, grad: torch.Tensor, post=None, wait=None) -> None:
        """Bucket k of the flat gradient buffer `grad` is final on the current stream: start its
        all-reduce (SUM) on the side stream, then run ``post(a, b)`` there once the reduced values are
        in place (the overlapped optimizer update of that parameter range)."""
        if not self.active and post is None:
            return
        a, b = self.buckets[k]

        def run():
            if self.active:
                import torch.distributed as dist
                work = dist.all_reduce(grad[a:b], group=self.pg, async_op=True)
                if post is not None:
                    work.wait()  # the side stream waits for the collective; no host synchronisation
                else:
                    self._works.append(work)
            if post is not None:
                post(a, b)
        self.enqueue(grad, run, k, wait)

    def finish(self, grad: torch.Tensor) -> None:
        """Make the current stream wait for every outstanding bucket (no host synchronisation)."""
        for w in self._works:
            w.wait()
        self._works = []
        if grad.is_cuda and self._stream is not None:
            torch.cuda.current_stream(grad.device).wait_stream(self._stream)
