"""Data-parallel synchronisation for the fused training step (one process per GPU).

The reference trains on one device (src/main.py:40-43) and has no collective; the build adds pure
data parallelism:

1. Loss normalisation.  The reference LM loss is a mean over the valid (!= -100) shifted labels of the
   whole batch and the emotion loss a mean over the batch (src/model.py:704-713).  Each rank therefore
   divides its local sums by the GLOBAL valid-label count (all-reduced before the forward) and by the
   global batch, so the SUM over ranks of local gradients equals the gradient of the concatenated
   global batch on one device.
2. Gradient reduction (SUM) of contiguous buckets of the flat gradient buffer, launched on a side
   stream as soon as the backward stage that finalises each bucket has been enqueued, so RCCL over
   xGMI overlaps the remaining backward.  The last bucket (caption K/V + wpe + wte) is final only after
   the embedding backward and cannot overlap.
3. Exchange precision (``grad_comm``): "bf16" (default) moves bf16 gradients and accumulates in fp32 —
   an all-to-all of bf16 chunks (rank r receives chunk r of every rank), an fp32 sum of the world
   copies of its chunk in rank order (ergm_chunk_sum_bf16, deterministic) rounded once to bf16, an
   all-gather of the reduced bf16 chunks, cast back into the fp32 gradient buffer: half the bytes of
   an fp32 all-reduce (2·(N−1)/N · 2 B per parameter), one rounding of the summed gradient, the same
   result on every rank.  "fp32": a plain fp32 all-reduce.  ERGM_DP_GRAD selects (default bf16).

Works with any torch.distributed backend: "nccl" (= RCCL on ROCm) on GPUs, "gloo" for CPU tests (CPU
tensors take torch ops for the cast and the chunk sum: that is the host-logic test path; GPU tensors
always run the HIP kernels).
"""
from __future__ import annotations

import ctypes as C
import os
from typing import List, Optional, Tuple

import torch


class DPSync:
    def __init__(self, process_group=None, buckets: Optional[List[Tuple[int, int]]] = None,
                 grad_comm: Optional[str] = None):
        self.pg = process_group
        self.buckets = buckets or []
        self._works: List = []
        self._stream = None
        self._events: List = []
        self.grad_comm = grad_comm or os.environ.get("ERGM_DP_GRAD", "bf16")
        if self.grad_comm not in ("bf16", "fp32"):
            raise ValueError(f"grad_comm must be 'bf16' or 'fp32' (got {self.grad_comm!r})")
        self._pool = None          # bf16 exchange buffers, reused in stream order by every reduction
        self.bytes_per_step = 0    # gradient bytes this rank sent in the last backward (bench report)

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
        self.bytes_per_step = 0

    def _buffers(self, chunk: int, dev) -> Tuple[torch.Tensor, ...]:
        W = self.world
        need = W * chunk
        if self._pool is None or self._pool[0].numel() < need or self._pool[0].device != dev:
            send = torch.zeros(need, dtype=torch.bfloat16, device=dev)
            self._pool = (send, torch.empty_like(send), torch.empty_like(send))
        send, recv, gath = self._pool
        return send[:need], recv[:need], gath[:need]

    def reduce_(self, t: torch.Tensor) -> None:
        """In place on the current stream: t = Σ over ranks of t (SUM), no host synchronisation."""
        if not self.active:
            return
        import torch.distributed as dist
        W, n = self.world, t.numel()
        if self.grad_comm == "fp32" or t.dtype != torch.float32:
            self.bytes_per_step += 2 * (W - 1) * n * t.element_size() // W
            dist.all_reduce(t, group=self.pg, async_op=True).wait()
            return
        chunk = -(-(-(-n // W)) // 8) * 8
        send, recv, gath = self._buffers(chunk, t.device)
        mine = gath.view(W, chunk)[self.rank]
        self.bytes_per_step += 2 * (W - 1) * chunk * 2
        if t.is_cuda:
            from . import _lib as L
            st = C.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)
            if W * chunk > n:
                send[n:].zero_()
            L.call("ergm_cast_bf16", C.c_void_p(t.data_ptr()), C.c_void_p(send.data_ptr()), n, st)
            dist.all_to_all_single(recv, send, group=self.pg, async_op=True).wait()
            L.call("ergm_chunk_sum_bf16", C.c_void_p(recv.data_ptr()), W, chunk, C.c_void_p(mine.data_ptr()), st)
            dist.all_gather_into_tensor(gath, mine, group=self.pg, async_op=True).wait()
            L.call("ergm_cast_f32", C.c_void_p(gath.data_ptr()), C.c_void_p(t.data_ptr()), n, st)
        else:  # gloo on CPU tensors (host-logic tests): the same arithmetic with torch ops
            send.zero_()
            send[:n] = t.to(torch.bfloat16)
            dist.all_to_all_single(recv, send, group=self.pg)
            mine.copy_(recv.view(W, chunk).float().sum(0).to(torch.bfloat16))
            dist.all_gather_into_tensor(gath, mine.clone(), group=self.pg)
            t.copy_(gath[:n].float())

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
            self.reduce_(grad[a:b])  # the side stream waits for the collectives; no host synchronisation
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
