"""Drop-in ``GPT2LMHeadModel`` of ERGM, running the fused HIP training step on MI355X.

Mirrors the reference interface (src/model.py:599-737):

* ``GPT2LMHeadModel(config)`` with the reference's state_dict names (``transformer.h.{i}...``,
  tied ``lm_head.weight``, ``emotion_head.weight``) so checkpoints interchange;
* ``forward(input_ids, token_type_ids=, labels=, emotion_labels=, imgs=, auds=, caption_ids=)``
  (plus the build's aliases ``visual_feat=`` / ``audio_feat=``) returning an object with ``.loss``,
  ``.logits`` [B,S,V] and ``.emotion_logits`` [B,7] (``CausalLMOutputWithEmotionClassification``,
  src/model.py:48-60);
* ``loss.backward()`` fills the parameter gradients; ``torch.optim.AdamW(model.parameters())`` works
  unchanged, and ``ergm_amd.optim.FusedAdamW`` runs the same update as one HIP kernel.

Storage (see params.py): one fp32 ``nn.Parameter`` holding every weight, a bf16 shadow read by the
MFMA GEMMs, one fp32 gradient buffer.  The whole forward is one native call and the backward three
native stages per step (ergm_model_* in include/ergm_hip.h); there is no CPU fallback.

Dropout follows nn.Module semantics: in ``train()`` mode (the default, as the reference trainer runs,
src/main.py:129) the attention-probability, residual-branch and embedding dropouts of the config
(``attn_pdrop`` / ``resid_pdrop`` / ``embd_pdrop``, 0.1 like GPT2Config / the "gpt2" checkpoint) are
applied with counter-based masks (include/ergm_hip.h ergm_dropout); ``eval()`` disables them.  The
masks are drawn from ``torch``'s default generator at construction (``torch.manual_seed`` makes a run
reproducible) and advance with every training forward.

``logits`` are fp32 and differentiable like the reference's (cast on first access from the bf16 GEMM
output, ``logits_bf16``; a loss built on them back-propagates).  Differences from the reference, by
design: ``emotion_logits`` are not differentiable (the trainer back-propagates ``loss``); the KV-cache /
``past_key_values``, ``attention_mask``, ``head_mask``, ``inputs_embeds`` and ``output_attentions``
paths are not part of the training hot path and raise ``NotImplementedError``.  A second training
forward of the same shape before the first one's backward raises in that backward (one set of saved
activations per shape).
"""
from __future__ import annotations

import ctypes as C
import os
import warnings
import weakref
from collections import OrderedDict
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import torch
import torch.nn as nn

from . import ops
from .config import ERGMConfig, NUM_EMOTIONS
from .params import build_layout, state_dict_names
from .runtime import ModelRunner


class _LazyLogits:
    """Descriptor of ``CausalLMOutputWithEmotionClassification.logits`` (a dataclass field): a value given to the
    constructor (``logits=...``, as the reference builds it) is returned as is; otherwise the fp32 cast of
    ``logits_bf16`` is made on first access, so a training step that never reads the logits pays nothing."""

    def __get__(self, obj, objtype=None):
        if obj is None:
            return None  # the field's default
        v = obj.__dict__.get("_logits32")
        if v is None and obj.__dict__.get("logits_bf16") is not None:
            v = obj.logits_bf16.float()
            obj.__dict__["_logits32"] = v
        return v

    def __set__(self, obj, value):
        obj.__dict__["_logits32"] = value


@dataclass
class CausalLMOutputWithEmotionClassification:
    """src/model.py:48-60 (fields the training path produces, in the reference's order).

    ``logits`` is fp32 [B,S,V] and differentiable like the reference's (src/model.py:698,731): it is the
    compute-dtype (bf16) GEMM output ``logits_bf16`` cast on first access (or the tensor passed as ``logits=``);
    a loss built on it back-propagates through the fused backward (its gradient is added to the cross-entropy's
    before the LM-head backward GEMMs)."""
    loss: Optional[torch.Tensor] = None
    logits: Optional[torch.Tensor] = _LazyLogits()
    emotion_logits: Optional[torch.Tensor] = None
    past_key_values: Optional[tuple] = None
    hidden_states: Optional[tuple] = None
    attentions: Optional[tuple] = None
    cross_attentions: Optional[tuple] = None
    logits_bf16: Optional[torch.Tensor] = None    # build extra: [B,S,V] view of the bf16 GEMM output
    loss_lm: Optional[torch.Tensor] = None        # build extra: the LM part (PPL = exp(loss_lm))
    loss_emotion: Optional[torch.Tensor] = None   # build extra: the emotion CE part

    def __getitem__(self, i):
        return (self.loss, self.logits, self.emotion_logits)[i]


def _as_config(config) -> ERGMConfig:
    if isinstance(config, ERGMConfig):
        return config
    g = lambda k, d=None: getattr(config, k, d)  # noqa: E731  (transformers GPT2Config)
    return ERGMConfig(vocab_size=g("vocab_size"), n_embd=g("n_embd"), n_layer=g("n_layer"), n_head=g("n_head"),
                      n_positions=g("n_positions", 1024), n_inner=g("n_inner"),
                      layer_norm_epsilon=g("layer_norm_epsilon", 1e-5),
                      initializer_range=g("initializer_range", 0.02), feat_dim=g("feat_dim"),
                      attn_pdrop=g("attn_pdrop", 0.1), resid_pdrop=g("resid_pdrop", 0.1),
                      embd_pdrop=g("embd_pdrop", 0.1))


# ---- the fused training step as PyTorch custom ops ------------------------------------------------
# ``ergm::train_step`` (one native forward: loss parts, logits, emotion logits) and
# ``ergm::train_step_backward`` (the native backward stages: the flat parameter gradient) are
# registered with torch.library so autograd and torch.compile treat them as opaque operators
# (register_fake gives their shapes; register_autograd connects them).  The model and its per-shape
# runner are named by integers (a model handle and the runner's shape key), because custom ops take
# tensors and plain values only.
_MODELS: "weakref.WeakValueDictionary[int, GPT2LMHeadModel]" = weakref.WeakValueDictionary()


def _model_of(handle: int) -> "GPT2LMHeadModel":
    m = _MODELS.get(handle)
    if m is None:
        raise RuntimeError(f"ergm: model handle {handle} is gone")
    return m


@torch.library.custom_op("ergm::train_step", mutates_args=())
def _train_step(flat: torch.Tensor, ids: torch.Tensor, tt: Optional[torch.Tensor], cap_ids: torch.Tensor,
                vis: Optional[torch.Tensor], aud: Optional[torch.Tensor], labels: Optional[torch.Tensor],
                emo_labels: Optional[torch.Tensor], handle: int,
                key: List[int]) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    model = _model_of(handle)
    runner = model._runners[tuple(key)]
    logits, emo, loss = runner.forward(ids, tt, cap_ids, vis, aud, labels, emo_labels, train=True,
                                       dropout=model._next_dropout())
    return loss, logits, emo


@_train_step.register_fake
def _(flat, ids, tt, cap_ids, vis, aud, labels, emo_labels, handle, key):
    B, S = ids.shape
    Vp = _model_of(handle).layout.vocab_pad
    return (flat.new_empty(3), flat.new_empty(B * S, Vp, dtype=torch.bfloat16), flat.new_empty(B, NUM_EMOTIONS))


@torch.library.custom_op("ergm::train_step_backward", mutates_args=())
def _train_step_backward(flat: torch.Tensor, grad_loss: torch.Tensor, grad_logits: Optional[torch.Tensor], handle: int,
                         key: List[int]) -> torch.Tensor:
    """Gradient of the flat parameter buffer for the runner's last training forward (fresh tensor);
    ``grad_logits`` (bf16 [B*S, Vp] or None) is a gradient on the returned logits."""
    model = _model_of(handle)
    model._runners[tuple(key)].backward(grad_loss, grad_logits=grad_logits)
    return model.grad_buf.clone()


@_train_step_backward.register_fake
def _(flat, grad_loss, grad_logits, handle, key):
    return torch.empty_like(flat)


_warned_compiled_logits = [False]


def _train_step_setup(ctx, inputs, output):
    handle, key = inputs[8], inputs[9]
    ctx.handle, ctx.key = handle, key
    model = _MODELS.get(handle)
    ctx.fwd_id = model._runners[tuple(key)].fwd_count if model is not None and not _compiling(output[0]) else -1
    ctx.mark_non_differentiable(output[2])
    if model is not None and _compiling(output[0]) and not model.compiled_logits_grad:
        ctx.mark_non_differentiable(output[1])
        if not _warned_compiled_logits[0]:  # a loss on the compiled logits would silently lose its term
            _warned_compiled_logits[0] = True
            warnings.warn("ergm: under torch.compile the returned logits are non-differentiable (a loss term built on "
                          "them contributes no gradient); set GPT2LMHeadModel.compiled_logits_grad = True BEFORE "
                          "compiling to differentiate through them (the flag is read at trace time)", stacklevel=2)
    ctx.set_materialize_grads(False)
    ctx.save_for_backward(inputs[0])


def _compiling(t: Optional[torch.Tensor] = None) -> bool:
    """Under torch.compile: Dynamo tracing, or AOTAutograd tracing the backward with fake tensors."""
    if bool(getattr(torch.compiler, "is_compiling", lambda: False)()):
        return True
    if t is not None:
        from torch._subclasses.fake_tensor import is_fake
        return bool(is_fake(t))
    return False


def _train_step_grad(ctx, grad_loss, grad_logits, grad_emo):
    nones = (None,) * 9
    if grad_loss is None and grad_logits is None:
        return (None,) + nones
    if grad_loss is None:  # only the logits were differentiated: the loss part contributes nothing
        gl = torch.zeros(1, dtype=torch.float32, device=grad_logits.device)
    else:
        gl = grad_loss.reshape(-1)[2:3] if grad_loss.numel() == 3 else grad_loss.reshape(1)
        gl = gl.float().contiguous()
    if grad_logits is not None:
        grad_logits = grad_logits.to(torch.bfloat16).contiguous()
    if _compiling(gl):  # traced by AOTAutograd: the opaque backward op, its output accumulated by autograd
        # (AOTAutograd hands every differentiable output a tangent, zeros when the loss ignores the logits)
        flat, = ctx.saved_tensors
        return (torch.ops.ergm.train_step_backward(flat, gl, grad_logits, ctx.handle, ctx.key),) + nones
    model = _model_of(ctx.handle)
    runner = model._runners[tuple(ctx.key)]
    if runner.fwd_count != ctx.fwd_id:
        raise RuntimeError("another forward of the same (batch, seq) shape ran after this training forward and "
                           "overwrote its saved activations: call backward() before the next forward of the "
                           "shape (e.g. backward per micro-batch for gradient accumulation)")
    # eager: the native backward writes straight into the flat gradient buffer, installed as
    # flat.grad (no 600 MB accumulate pass); the flat input's returned gradient is None
    flat = model.flat
    if flat.grad is None:
        post = native = None
        opt = model._overlap_opt
        if opt is not None:  # per-bucket AdamW, overlapped with backward
            if runner.dp.active or runner.compact_lookup:
                post = opt._backward_hook(flat, model)   # after each bucket's exchange (Python, comm stream)
            else:
                native = opt._native_desc(flat, model)   # scheduled by the executor
        runner.backward(gl, post, native, grad_logits)  # writes model.grad_buf
        if native is not None and native.defer:
            model._deferred = runner                 # its block updates are still running (next forward waits)
        flat.grad = model.grad_buf
    elif flat.grad.data_ptr() == model.grad_buf.data_ptr():
        # accumulate semantics when the caller did not zero the gradient
        tmp = model._grad_tmp()
        tmp.copy_(model.grad_buf)                    # the gradient accumulated so far
        runner.backward(gl, grad_logits=grad_logits)  # overwrites grad_buf with this backward's
        ops.axpy(tmp, model.grad_buf)
    else:
        runner.backward(gl, grad_logits=grad_logits)
        ops.axpy(model.grad_buf, flat.grad)
    return (None,) + nones


torch.library.register_autograd("ergm::train_step", _train_step_grad, setup_context=_train_step_setup)


class GPT2LMHeadModel(nn.Module):
    num_emotions = NUM_EMOTIONS
    # Under torch.compile AOTAutograd hands every differentiable output a tangent — zeros for logits the loss
    # ignores — and the backward would then add a T x vocab bf16 zero gradient into dlogits (~200 MB of traffic at
    # C2).  The compiled step therefore returns non-differentiable logits unless this is set; eager mode keeps them
    # differentiable either way (no tangent is materialised there).
    compiled_logits_grad = False

    def __init__(self, config, device=None, process_group=None):
        super().__init__()
        cfg = _as_config(config)
        cfg.validate()
        if cfg.head_dim != 64:
            raise ValueError(f"head_dim must be 64 for the fused attention kernels (got {cfg.head_dim})")
        self.config = cfg
        dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.layout = build_layout(cfg.vocab_size, cfg.n_embd, cfg.n_layer, cfg.inner, cfg.n_positions,
                                   feat_dim=cfg.feat_dim)
        n = self.layout.total
        self.flat = nn.Parameter(torch.zeros(n, dtype=torch.float32, device=dev))
        self.register_buffer("flat_b16", torch.zeros(n, dtype=torch.bfloat16, device=dev), persistent=False)
        self.grad_buf = torch.zeros(n, dtype=torch.float32, device=dev)
        self._tmp = None
        self._runners: Dict[tuple, ModelRunner] = {}
        self._train_metrics = None  # set_train_metrics
        self._b16_version = -1
        self._overlap_opt = None
        self._deferred = None  # runner whose deferred optimizer updates no forward has waited for yet
        self._force_compact_lookup = False  # tests: the data-parallel wte path in one process
        self.process_group = process_group
        self._handle = id(self)
        _MODELS[self._handle] = self
        # dropout mask stream: seed from torch's default generator (torch.manual_seed makes it reproducible),
        # offset = training forwards so far; under data parallelism rank 0's seed is broadcast so every rank
        # draws the masks one process would draw for the concatenated batch (rows are global)
        self.reseed_dropout()
        self.init_weights()

    def reseed_dropout(self) -> None:
        """Draw the dropout mask stream's seed from torch's default generator and restart its forward count:
        after ``torch.manual_seed(s)`` the following training forwards draw the same masks as after any other
        ``torch.manual_seed(s)`` (the reference seeds torch at every ``train()`` start, src/main.py:124,284-289,
        which fixes its dropout masks).  Under data parallelism rank 0's seed is broadcast (collective)."""
        self._drop_seed = int(torch.randint(0, 2 ** 62, (1,)).item())
        pg = self.process_group
        if pg is not None:
            import torch.distributed as dist
            if dist.get_world_size(pg) > 1:
                bdev = self.flat.device if dist.get_backend(pg) == "nccl" else torch.device("cpu")
                t = torch.tensor([self._drop_seed], dtype=torch.int64, device=bdev)
                dist.broadcast(t, src=dist.get_global_rank(pg, 0), group=pg)
                self._drop_seed = int(t.item())
        self._drop_offset = 0

    # ---- parameters / state_dict ---------------------------------------------------------
    def view(self, name: str, t: Optional[torch.Tensor] = None) -> torch.Tensor:
        v = self.layout.views[name]
        t = self.flat.data if t is None else t
        return t.as_strided(v.shape, v.stride, v.offset)

    def init_weights(self, seed: Optional[int] = None) -> None:
        """``_init_weights`` (src/model.py:359-375): N(0, 0.02) matrices and embeddings, c_proj
        N(0, 0.02/sqrt(2L)), LayerNorm 1/0, biases 0; padding rows zero."""
        cfg = self.config
        g = torch.Generator(device="cpu")
        g.manual_seed(0 if seed is None else seed)
        sd = {}
        for name in state_dict_names(self.layout):
            if name == "lm_head.weight":
                continue
            shape = self.layout.views[name].shape
            if name.endswith("c_proj.weight"):
                t = torch.randn(shape, generator=g) * (cfg.initializer_range / (2 * cfg.n_layer) ** 0.5)
            elif len(shape) == 2:
                t = torch.randn(shape, generator=g) * cfg.initializer_range
            elif name.endswith("ln_1.weight") or name.endswith("ln_2.weight") or "ln_cross_attn.weight" in name \
                    or name.endswith("ln_f.weight"):
                t = torch.ones(shape)
            else:
                t = torch.zeros(shape)
            sd[name] = t
        self.load_state_dict(sd, strict=False)

    def state_dict(self, *args, destination=None, prefix="", keep_vars=False):
        self.flush_deferred_()
        if self.master_sharded:
            raise RuntimeError("the sharded optimizer update (ZeRO-1, ERGM_DP_ZERO=1) left this rank's fp32 master "
                               "valid only in its own chunks: call model.consolidate_() on EVERY rank (a collective) "
                               "before state_dict()")
        out = OrderedDict() if destination is None else destination
        for name in state_dict_names(self.layout):
            src = "transformer.wte.weight" if name == "lm_head.weight" else name
            out[prefix + name] = self.view(src).detach()
        return out

    @torch.no_grad()
    def load_state_dict(self, state_dict, strict: bool = True, assign: bool = False):
        names = set(state_dict_names(self.layout))
        missing = [k for k in names if k not in state_dict and k != "lm_head.weight"]
        unexpected = [k for k in state_dict if k not in names]
        if strict and (missing or unexpected):
            raise RuntimeError(f"Error(s) in loading state_dict: missing {missing}, unexpected {unexpected}")
        for k, v in state_dict.items():
            if k not in names or k == "lm_head.weight":
                continue
            dst = self.view(k)
            if tuple(v.shape) != tuple(dst.shape):
                raise RuntimeError(f"size mismatch for {k}: {tuple(v.shape)} vs {tuple(dst.shape)}")
            dst.copy_(v.to(dst.device, torch.float32))
        if "lm_head.weight" in state_dict and "transformer.wte.weight" not in state_dict:
            self.view("transformer.wte.weight").copy_(state_dict["lm_head.weight"])
        self.refresh_bf16()
        for r in self._runners.values():  # every rank now holds the full master (the moments stay sharded)
            r.dp.master_sharded.clear()
        return torch.nn.modules.module._IncompatibleKeys(missing, unexpected)

    def flush_deferred_(self) -> None:
        """Order the current stream after the optimizer's deferred block updates (FusedAdamW(defer=True)):
        call before reading the parameters other than through a forward (which waits by itself)."""
        r, self._deferred = self._deferred, None
        if r is not None:
            from . import _lib as L
            L.check(r.lib.ergm_model_optimizer_join(r.plan, C.c_void_p(torch.cuda.current_stream(r.dev).cuda_stream)),
                    "ergm_model_optimizer_join")

    @torch.no_grad()
    def consolidate_(self) -> None:
        """Data parallel with the sharded optimizer update (ZeRO-1, ergm_amd/dist.py): all-gather the
        owners' chunks of the fp32 master, the gradient and the overlapped optimizer's moments, so every
        rank holds the full values (before a checkpoint, state_dict() or a non-overlapped update).
        Collective: every rank must call it.  No-op when nothing is sharded."""
        rs = [r for r in self._runners.values() if r.dp.sharded]
        if not rs:
            return
        ranges = set().union(*(r.dp.sharded for r in rs))
        ts = [self.flat.data, self.grad_buf]
        opt = self._overlap_opt
        st = opt.state.get(self.flat) if opt is not None else None
        if st:
            ts += [st["exp_avg"], st["exp_avg_sq"]]
        rs[0].dp.consolidate_(ts, ranges)
        for r in rs:
            r.dp.sharded.clear()
            r.dp.master_sharded.clear()

    @property
    def sharded(self) -> bool:
        """True while the gradient / optimizer moments of some parameter range are only valid on their owner
        rank (see consolidate_)."""
        return any(r.dp.sharded for r in self._runners.values())

    @property
    def master_sharded(self) -> bool:
        """True while the fp32 master of some parameter range is only valid on its owner rank."""
        return any(r.dp.master_sharded for r in self._runners.values())

    @torch.no_grad()
    def refresh_bf16(self) -> None:
        self.flush_deferred_()
        ops.cast_bf16(self.flat.data, self.flat_b16)
        self._b16_version = self.flat._version

    def _grad_tmp(self) -> torch.Tensor:
        if self._tmp is None:
            self._tmp = torch.zeros_like(self.grad_buf)
        return self._tmp

    def get_input_embeddings(self):
        return self.view("transformer.wte.weight")

    def get_output_embeddings(self):
        return self.view("transformer.wte.weight")

    def num_parameters(self) -> int:
        """Reference parameter count (tied lm_head counted once, no padding)."""
        return sum(self.layout.views[k].numel for k in state_dict_names(self.layout) if k != "lm_head.weight")

    # ---- forward ---------------------------------------------------------------------------
    def _next_dropout(self):
        """(attn_p, resid_p, embd_p, seed, offset) of the next training forward, None when every
        probability is 0 or the module is in eval mode."""
        c = self.config
        if not self.training or not (c.attn_pdrop or c.resid_pdrop or c.embd_pdrop):
            return None
        self._drop_offset += 1
        return (float(c.attn_pdrop), float(c.resid_pdrop), float(c.embd_pdrop), self._drop_seed, self._drop_offset)

    def _runner(self, B, S, vis_rows, has_feat) -> ModelRunner:
        key = (B, S, vis_rows, int(bool(has_feat)))
        r = self._runners.get(key)
        if r is None:
            r = ModelRunner(self.layout, self.config, self.flat.data, self.flat_b16, self.grad_buf, B, S, vis_rows,
                            has_feat, self.process_group)
            if self._force_compact_lookup:
                r.force_compact_lookup()
            if self._train_metrics is not None:
                r.set_metrics(*self._train_metrics)
            self._runners[key] = r
        return r

    def set_train_metrics(self, loss_acc: Optional[torch.Tensor], correct: Optional[torch.Tensor] = None) -> None:
        """Accumulate the trainer's per-step metrics on the device (src/main.py:158-169): every training
        forward adds its loss to ``loss_acc[0]``, its LM loss to ``loss_acc[1]`` (fp32, 2 elements) and its
        emotion argmax hits to ``correct`` (int64, 1 element), inside the loss finalisation — the same
        numbers as ``loss_acc += (out.loss, out.loss_lm)`` and ``correct += (argmax == labels).sum()`` with
        no extra launches.  ``None`` turns it off."""
        if loss_acc is not None:
            if loss_acc.dtype != torch.float32 or loss_acc.numel() < 2 or not loss_acc.is_contiguous():
                raise ValueError("loss_acc must be a contiguous fp32 tensor of 2 elements")
            if correct is not None and (correct.dtype != torch.int64 or correct.numel() < 1):
                raise ValueError("correct must be an int64 tensor of 1 element")
        self._train_metrics = None if loss_acc is None else (loss_acc, correct)
        for r in self._runners.values():
            r.set_metrics(loss_acc, correct if loss_acc is not None else None)

    def forward(self, input_ids=None, past_key_values=None, attention_mask=None, token_type_ids=None,
                position_ids=None, head_mask=None, inputs_embeds=None, encoder_hidden_states=None,
                encoder_attention_mask=None, labels=None, emotion_labels=None, use_cache=None,
                output_attentions=None, output_hidden_states=None, return_dict=None, imgs=None, auds=None,
                caption_ids=None, visual_feat=None, audio_feat=None):
        for name, val in (("past_key_values", past_key_values), ("attention_mask", attention_mask),
                          ("position_ids", position_ids), ("head_mask", head_mask), ("inputs_embeds", inputs_embeds),
                          ("encoder_hidden_states", encoder_hidden_states),
                          ("encoder_attention_mask", encoder_attention_mask)):
            if val is not None:
                raise NotImplementedError(f"{name} is not supported by the fused training path")
        if output_attentions or output_hidden_states:
            raise NotImplementedError("output_attentions / output_hidden_states are not supported")
        if input_ids is None:
            raise ValueError("You have to specify either input_ids or inputs_embeds")
        if caption_ids is None:
            # src/model.py:521 reads caption_embeds unconditionally: the reference cannot run without it
            raise ValueError("caption_ids is required (the reference forward reads caption embeddings in every block)")
        if imgs is not None and visual_feat is None and torch.is_tensor(imgs) and imgs.dim() == 2:
            # the reference adds imgs[i][0] to position 0 (src/model.py:497): for a 2-D [B, E] tensor that
            # is the SCALAR imgs[i, 0], broadcast over the embedding (a [B, Tv, E] tensor gives row 0, the
            # pooled vector; visual_feat= [B, E] is the build's vector form)
            imgs = imgs[:, :1].expand(imgs.shape[0], self.layout.Fd).unsqueeze(1)
        vis = visual_feat if visual_feat is not None else imgs
        aud = audio_feat if audio_feat is not None else auds
        if (vis is None) != (aud is None):
            raise ValueError("imgs/visual_feat and auds/audio_feat must be given together (src/model.py:495-498)")
        dev = self.flat.device
        B, S = input_ids.shape
        Fd = self.layout.Fd

        def dv(t, dtype):
            return None if t is None else t.to(dev, dtype, non_blocking=True).contiguous()
        ids, tt, cap = dv(input_ids, torch.int64), dv(token_type_ids, torch.int64), dv(caption_ids, torch.int64)
        if tuple(cap.shape) != (B, S):
            raise ValueError(f"caption_ids must have the text shape {(B, S)} (src/model.py:461), got {tuple(cap.shape)}")
        if tt is not None and tuple(tt.shape) != (B, S):
            raise ValueError("token_type_ids must match input_ids")
        V = self.config.vocab_size
        for name, t, hi in (("labels", labels, V), ("emotion_labels", emotion_labels, self.num_emotions)):
            if t is not None and not t.is_cuda and t.numel():  # host labels: torch's range check, free here
                bad = (t != -100) & ((t < 0) | (t >= hi))
                if bool(bad.any()):
                    raise IndexError(f"{name}: target {int(t[bad][0])} is out of bounds (classes: {hi})")
        lab = dv(labels, torch.int64)
        emo_lab = dv(emotion_labels, torch.int64)
        vis_rows = 0
        if vis is not None:
            vis = dv(vis, torch.float32)
            aud = dv(aud, torch.float32)
            if vis.dim() == 2:
                vis = vis.unsqueeze(1)
            if vis.shape[0] != B or vis.shape[-1] != Fd or tuple(aud.shape) != (B, Fd):
                raise ValueError(f"visual [B,Tv,{Fd}] / audio [B,{Fd}] features expected, got {tuple(vis.shape)} / "
                                 f"{tuple(aud.shape)}")
            vis_rows = vis.shape[1]
        if S > self.config.n_positions:
            raise ValueError(f"sequence length {S} exceeds n_positions {self.config.n_positions}")
        if self.flat._version != self._b16_version:
            self.refresh_bf16()  # weights changed outside FusedAdamW (e.g. torch.optim.AdamW)
        runner = self._runner(B, S, vis_rows, vis is not None)
        if self._deferred is not None:  # the runner's own forward waits per block; another runner must join
            if self._deferred is not runner:
                self.flush_deferred_()
            self._deferred = None
        V, Vp = self.config.vocab_size, self.layout.vocab_pad
        if torch.is_grad_enabled() and self.flat.requires_grad and (lab is not None or emo_lab is not None):
            loss3, logits, emo = torch.ops.ergm.train_step(self.flat, ids, tt, cap, vis, aud, lab, emo_lab, self._handle,
                                                           list(runner.key))
        else:
            logits, emo, loss3 = runner.forward(ids, tt, cap, vis, aud, lab, emo_lab, train=False)
        out = CausalLMOutputWithEmotionClassification(
            logits_bf16=logits.view(B, S, Vp)[:, :, :V], emotion_logits=emo)
        if loss3 is not None:
            out.loss = loss3[2] if lab is not None or emo_lab is not None else None
            out.loss_lm = loss3[0].detach() if lab is not None else None
            out.loss_emotion = loss3[1].detach() if emo_lab is not None else None
        return out


FusedGPT2LMHead = GPT2LMHeadModel
