"""Native runner: binds the flat parameter buffers and a caller-owned workspace to one
``ergm_model_plan`` (per batch/sequence shape) and drives the C-ABI forward/backward stages.

Data parallelism (one process per GPU, ``torch.distributed`` with backend "nccl" = RCCL over xGMI):
before the forward the local count of valid LM labels is all-reduced so every rank normalises by the
GLOBAL count (and the emotion loss by the global batch) — summed gradients then equal the
single-process gradient of the concatenated global batch.  During backward each
finished gradient bucket (a contiguous range of the flat gradient buffer) is all-reduced on a side
stream while later blocks are still being differentiated.
"""
from __future__ import annotations

import ctypes as C
import time
from typing import Optional

import torch

from . import _lib as L
from .dist import DPSync
from .params import Layout, dp_buckets, master_read_ranges


def _p(t: Optional[torch.Tensor]):
    return None if t is None else C.c_void_p(t.data_ptr())


class ModelRunner:
    def __init__(self, layout: Layout, cfg, flat: torch.Tensor, flat_b16: torch.Tensor, grad: torch.Tensor,
                 B: int, S: int, vis_rows: int, has_features: bool, process_group=None):
        self.layout, self.cfg = layout, cfg
        self.B, self.S = B, S
        self.key = (B, S, vis_rows, int(bool(has_features)))  # the model's runner key
        self.dev = flat.device
        self.lib = L.load()
        E, Lyr = layout.E, layout.L
        self.dims = L.ModelDims(vocab=layout.vocab, vocab_pad=layout.vocab_pad, n_embd=E, n_layer=Lyr,
                                n_head=cfg.n_head, n_inner=layout.F, n_positions=layout.P, batch=B, seq=S,
                                eps=cfg.layer_norm_epsilon, has_features=int(has_features),
                                ld_vis=vis_rows * layout.Fd if has_features else 0, feat_dim=layout.Fd,
                                fp8=int(bool(getattr(cfg, "fp8", False))))
        ws_bytes = self.lib.ergm_model_workspace_size(C.byref(self.dims))
        self.workspace = torch.empty(ws_bytes, dtype=torch.uint8, device=self.dev)
        v = layout.views
        fp, bp, gp = flat.data_ptr(), flat_b16.data_ptr(), grad.data_ptr()

        def f32(name):
            return C.c_void_p(fp + 4 * v[name].offset)

        def b16(name):
            return C.c_void_p(bp + 2 * v[name].offset)

        def g32(name):
            return C.c_void_p(gp + 4 * v[name].offset)

        prm = L.ModelParams()
        prm.wte, prm.wte_b = f32("__wte_pad"), b16("__wte_pad")
        prm.wpe = f32("transformer.wpe.weight")
        prm.ln_f_w, prm.ln_f_b = f32("transformer.ln_f.weight"), f32("transformer.ln_f.bias")
        prm.emo_w = f32("emotion_head.weight")
        prm.capkv_w_b, prm.capkv_b = b16("__capkv_w"), f32("__capkv_b")
        prm.capkv_w = f32("__capkv_w")
        prm.layer_f32 = C.c_void_p(fp + 4 * layout.layer_base[0])
        prm.layer_b16 = C.c_void_p(bp + 2 * layout.layer_base[0])
        prm.layer_stride = layout.layer_stride
        for i, o in enumerate(layout.layer_off):
            prm.layer_off[i] = o
        prm.g_wte, prm.g_wpe = g32("__wte_pad"), g32("transformer.wpe.weight")
        prm.g_ln_f_w, prm.g_ln_f_b = g32("transformer.ln_f.weight"), g32("transformer.ln_f.bias")
        prm.g_emo_w = g32("emotion_head.weight")
        prm.g_capkv_w, prm.g_capkv_b = g32("__capkv_w"), g32("__capkv_b")
        prm.g_layer = C.c_void_p(gp + 4 * layout.layer_base[0])
        if layout.Fd != E:
            prm.vproj_w_b, prm.vproj_b = b16("transformer.visual_proj.weight"), f32("transformer.visual_proj.bias")
            prm.aproj_w_b, prm.aproj_b = b16("transformer.audio_proj.weight"), f32("transformer.audio_proj.bias")
            prm.g_vproj_w, prm.g_vproj_b = g32("transformer.visual_proj.weight"), g32("transformer.visual_proj.bias")
            prm.g_aproj_w, prm.g_aproj_b = g32("transformer.audio_proj.weight"), g32("transformer.audio_proj.bias")
        self._params = prm  # keep alive
        plan = C.c_void_p()
        L.check(self.lib.ergm_model_create(C.byref(self.dims), C.byref(prm), _p(self.workspace), ws_bytes,
                                           C.byref(plan)), "ergm_model_create")
        self.plan = plan
        # the data-gradient chain never waits for the weight-gradient stream between blocks; the
        # consumers of each block's gradients (all-reduce, overlapped AdamW) wait for its mark instead
        self.per_stage_join = False
        L.check(self.lib.ergm_model_set_side_joins(self.plan, int(self.per_stage_join)), "ergm_model_set_side_joins")
        self.grad = grad
        self.shadow = flat_b16
        self.dp = DPSync(process_group, dp_buckets(layout))
        self.dp.set_master(flat, master_read_ranges(layout, bool(getattr(cfg, "fp8", False))))
        self.n_valid = torch.zeros(4, dtype=torch.int32, device=self.dev)  # [LM, emotion] valid-label counts
        self._inputs = None
        # every forward overwrites the activations saved for backward: the autograd bridge checks that
        # the forward it differentiates is still the runner's last one
        self.fwd_count = 0
        # rows of the tied wte the batch's lookups touch (written by every training forward)
        self.row_flags = torch.zeros(layout.vocab_pad, dtype=torch.uint8, device=self.dev)
        L.check(self.lib.ergm_model_set_row_flags(self.plan, _p(self.row_flags), layout.vocab_pad),
                "ergm_model_set_row_flags")
        # Data parallelism: the lookup part of the wte gradient is exchanged as a compact block of the
        # ranks' union of touched rows (ergm_model_set_lookup_compact); the dense LM-head part is
        # all-reduced early, during the block backward.  compact_lookup can be forced for testing.
        self.compact_lookup = self.dp.active
        self.host_sync_s = 0.0  # host time spent waiting for the compact row count (DP), diagnostics
        self._compact_ready = False
        if self.compact_lookup:
            self._setup_compact()

    def set_metrics(self, loss_acc: Optional[torch.Tensor], correct: Optional[torch.Tensor]) -> None:
        """Device-side trainer metrics of every training forward (ergm_model_set_metrics)."""
        self._metrics = (loss_acc, correct)  # keep alive
        L.check(self.lib.ergm_model_set_metrics(self.plan, _p(loss_acc), _p(correct)), "ergm_model_set_metrics")

    def _setup_compact(self):
        Vp, E = self.layout.vocab_pad, self.layout.E
        cap = min(Vp, self.dp.world * 3 * self.B * self.S)
        self.row_pos = torch.zeros(Vp, dtype=torch.int32, device=self.dev)
        self.row_count = torch.zeros(1, dtype=torch.int32, device=self.dev)
        self.row_count_host = torch.zeros(1, dtype=torch.int32).pin_memory()
        self.compact = torch.zeros(cap * E, dtype=torch.float32, device=self.dev)
        self._ev_count = torch.cuda.Event()
        self._ev_zero = L.HipEvent(sync=True)
        L.check(self.lib.ergm_model_set_lookup_compact(self.plan, _p(self.row_pos), _p(self.compact)),
                "ergm_model_set_lookup_compact")

    def force_compact_lookup(self):
        """Use the data-parallel compact lookup-gradient path even in one process (tests)."""
        if not self.compact_lookup:
            self.compact_lookup = True
            self._setup_compact()

    def _prepare_compact(self):
        """After a training forward (comm stream): union of touched rows over ranks, their numbering,
        the count (copied to the host, read at the end of the backward) and zeroed compact rows."""
        Vp, E, lib = self.layout.vocab_pad, self.layout.E, self.lib
        dp = self.dp

        def prep():
            st = torch.cuda.current_stream(self.dev).cuda_stream
            if dp.active:
                import torch.distributed as dist
                dist.all_reduce(self.row_flags, op=dist.ReduceOp.MAX, group=dp.pg, async_op=True).wait()
            L.check(lib.ergm_rows_scan(_p(self.row_flags), Vp, _p(self.row_pos), _p(self.row_count),
                                       C.c_void_p(st)), "ergm_rows_scan")
            self.row_count_host.copy_(self.row_count, non_blocking=True)
            self._ev_count.record()
            L.check(lib.ergm_rows_compact(_p(self.row_flags), _p(self.row_pos), Vp, E, _p(self.compact), None, 0,
                                          C.c_void_p(st)), "ergm_rows_compact")
            self._ev_zero.record(st)
        dp.enqueue(self.grad, prep, self.layout.L + 4)
        self._compact_ready = True

    def __del__(self):
        try:
            if getattr(self, "plan", None):
                self.lib.ergm_model_destroy(self.plan)
        except Exception:
            pass

    def _stream(self):
        return C.c_void_p(torch.cuda.current_stream(self.dev).cuda_stream)

    # ---- forward ------------------------------------------------------------------------
    def forward(self, ids, tt, cap_ids, vis, aud, labels, emo_labels, train: bool, dropout=None):
        """Returns (logits [B*S, Vp] bf16, emotion_logits [B, 7] f32, loss3 [3] f32 or None).
        ``dropout`` = (attn_p, resid_p, embd_p, seed, offset) for a training forward (None: no dropout)."""
        dev, B, S = self.dev, self.B, self.S
        s = self._stream()
        have_labels = labels is not None or emo_labels is not None
        if have_labels:
            from .config import NUM_EMOTIONS
            L.check(self.lib.ergm_count_valid(_p(labels), _p(emo_labels), B, S, self.layout.vocab, NUM_EMOTIONS,
                                              _p(self.n_valid), s), "ergm_count_valid")
            self.dp.reduce_count(self.n_valid[:2])
        self._inputs = (ids, tt, cap_ids, vis, aud, labels, emo_labels)  # keep alive through backward
        L.check(self.lib.ergm_model_set_inputs(self.plan, _p(ids), _p(tt), _p(cap_ids), _p(vis), _p(aud), _p(labels),
                                               _p(emo_labels), _p(self.n_valid) if have_labels else None),
                "ergm_model_set_inputs")
        pa, pr, pe, seed, offset = dropout if (dropout is not None and train) else (0.0, 0.0, 0.0, 0, 0)
        # rows counted from this rank's first global sample: DP ranks draw the masks one process would
        # draw for the concatenated batch (equal local batches)
        L.check(self.lib.ergm_model_set_dropout(self.plan, pa, pr, pe, seed & (2 ** 64 - 1), offset & 0xFFFFFFFF,
                                                self.dp.rank * B), "ergm_model_set_dropout")
        self.fwd_count += 1
        logits = torch.empty(B * S, self.layout.vocab_pad, dtype=torch.bfloat16, device=dev)
        emo = torch.empty(B, 7, dtype=torch.float32, device=dev)
        loss = torch.empty(3, dtype=torch.float32, device=dev) if (labels is not None or emo_labels is not None) else None
        L.check(self.lib.ergm_model_forward(self.plan, _p(logits), _p(emo), _p(loss), int(train), s),
                "ergm_model_forward")
        if train and self.compact_lookup:
            self._prepare_compact()
        return logits, emo, loss

    # ---- backward -----------------------------------------------------------------------
    def backward(self, grad_scale: Optional[torch.Tensor], post=None, native_opt=None,
                 grad_logits: Optional[torch.Tensor] = None) -> None:
        """Writes every parameter gradient into self.grad (overwrite, not accumulate).  With a
        process group, each bucket is all-reduced (SUM) on a side stream as soon as it is final.

        ``post(a, b, rows=None)`` (the overlapped optimizer) is run on that side stream for each final
        range.  Single-process, the tied wte is updated in two parts: the rows no lookup of this batch
        touched are final with the LM-head weight gradient (after block L-2's stage) and are updated
        while the remaining blocks are differentiated; the touched rows follow the embedding backward."""
        s = self._stream()
        lib = self.lib
        dp = self.dp
        dp.begin()
        # single process: the executor runs the per-bucket AdamW schedule itself (ergm_model_set_optimizer)
        L.check(lib.ergm_model_set_optimizer(self.plan, C.byref(native_opt) if native_opt is not None else None),
                "ergm_model_set_optimizer")
        if grad_logits is not None:  # a loss built on the returned logits (bf16 [B*S, Vp], kept alive until here)
            L.check(lib.ergm_model_set_logits_grad(self.plan, _p(grad_logits)), "ergm_model_set_logits_grad")
        L.check(lib.ergm_model_backward_head(self.plan, _p(grad_scale), s), "ergm_model_backward_head")
        Lyr, E, Vp = self.layout.L, self.layout.E, self.layout.vocab_pad
        compact = self.compact_lookup
        if compact and not self._compact_ready:
            raise RuntimeError("backward without a training forward")
        split_wte = compact or (post is not None and not dp.active)
        wa, wb = self.layout.seg["wte"]
        ca, cb = self.layout.seg["capwpe"]
        ka = Lyr + 1  # ordering-event keys beyond the buckets'

        def reduce(a, b):
            dp.reduce_(self.grad[a:b])

        def wte_lm_rows():  # dense LM-head part of g_wte (all rows), then the untouched rows' update
            if compact:
                reduce(wa, wb)
            if post is not None:
                post(wa, wb, rows=(E, self.row_flags, 0))

        def capwpe():
            if compact:
                dp.reduce_then(self.grad, ca, cb, post, self.shadow)
            elif post is not None:
                post(ca, cb)

        def wte_lookup_rows():  # lookup part of the touched rows, then their update
            if compact:
                t0 = time.perf_counter()
                self._ev_count.synchronize()  # recorded right after the forward: long complete
                self.host_sync_s += time.perf_counter() - t0
                n = int(self.row_count_host[0]) * E
                if dp.active and n:
                    dp.reduce_(self.compact[:n])
                st = torch.cuda.current_stream(self.dev).cuda_stream
                L.check(lib.ergm_rows_compact(_p(self.row_flags), _p(self.row_pos), Vp, E, _p(self.compact),
                                              C.c_void_p(self.grad.data_ptr() + 4 * wa), 1, C.c_void_p(st)),
                        "ergm_rows_compact")
            if post is not None:
                post(wa, wb, rows=(E, self.row_flags, 1))
        def stage(k):  # the consumer stream also waits for the executor's weight-gradient mark k
            if self.per_stage_join:
                return None
            return lambda st: L.check(lib.ergm_model_stage_wait(self.plan, k, C.c_void_p(st)), "ergm_model_stage_wait")
        # bucket i = (head +) block L-1-i; its data-gradient chain is done after stage L-1-i, its weight
        # gradients (side stream) at mark L-1-i; the LM-head part of wte at mark L+1 (ergm_hip.h)
        for i, l in enumerate(reversed(range(Lyr))):
            L.check(lib.ergm_model_backward_layer(self.plan, l, s), "ergm_model_backward_layer")
            if i >= 1:
                dp.bucket_ready(i - 1, self.grad, post, wait=stage(l + 1), shadow=self.shadow)
            if split_wte and i == 1:
                dp.enqueue(self.grad, wte_lm_rows, ka, wait=stage(Lyr + 1))
        if compact:
            self._ev_zero.wait(s.value)  # compact rows zeroed before the lookup sums land in them
            self._compact_ready = False
        L.check(lib.ergm_model_backward_embed(self.plan, s), "ergm_model_backward_embed")
        dp.bucket_ready(Lyr - 1, self.grad, post, shadow=self.shadow)
        if split_wte:
            if Lyr == 1:
                dp.enqueue(self.grad, wte_lm_rows, ka)
            dp.enqueue(self.grad, capwpe, ka + 1)
            dp.enqueue(self.grad, wte_lookup_rows, ka + 2)
        else:
            dp.bucket_ready(Lyr, self.grad, post)
        dp.finish(self.grad)
