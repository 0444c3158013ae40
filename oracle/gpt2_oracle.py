"""CPU fp32 oracle for ERGM's fused GPT-2 training step — TEST INFRASTRUCTURE ONLY.

This module is the checker, never the product: only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import it.  The product path (``ergm_amd``) never routes
through it and fails loudly when its HIP library is missing.

It restates, with plain PyTorch CPU fp32 ops and in the reference's arithmetic order, the hot path of
LovesickPatience/ERGM (``/root/reference``):

* ``GPT2Model.forward``          src/model.py:420-596 (embeddings :459-463,500-504, fusion :495-498,
                                 block loop :520-576, ln_f :578)
* ``GPT2Block.forward``          src/model.py:286-341 (pre-LN self-attn, cross-attn, MLP, 3 residuals)
* ``GPT2Attention.forward/_attn`` src/model.py:200-251, :119-148 (divide by sqrt(d), causal
                                 ``where(tril, w, finfo.min)``, softmax, PV; cross path: no causal mask,
                                 additive encoder mask of zeros :484-489)
* ``GPT2MLP.forward``            src/model.py:262-267 with transformers' ``NewGELUActivation``
                                 (gelu_new, tanh form) and ``Conv1D`` (``addmm(b, x, W)``, W is [in, out])
* ``GPT2LMHeadModel.forward``    src/model.py:654-737 (tied LM head :698, emotion head on the last
                                 token :700-701, LM CE on shifted logits + emotion CE :704-713)
* ``Manager.train`` step         src/main.py:147-156 (AdamW :68 with torch defaults, polynomial-decay
                                 schedule with warmup, power=2 :93-95)

Parity pinning: ``tests/golden/make_golden.py`` imports the reference model in the build container
(loader shim from SURVEY.md §8(c), no source edits) and checks this restatement against it; the
captured fixtures (``tests/golden/*.npz``) pin it on every later run, including on the GPU box where
the reference does not exist.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, Optional

import torch
import torch.nn.functional as F

NUM_EMOTIONS = 7  # src/model.py:607 (EMOTION_LIST in src/scripts/emotion_labels.py:9)


@dataclass
class OracleConfig:
    """GPT2Config fields read on the path (SURVEY §8(a) 'Types on the path')."""

    vocab_size: int = 50260
    n_embd: int = 768
    n_layer: int = 12
    n_head: int = 12
    n_positions: int = 1024
    layer_norm_epsilon: float = 1e-5
    initializer_range: float = 0.02
    n_inner: Optional[int] = None
    # Width of the pooled audio / visual features.  None (or == n_embd) is the reference model, which
    # adds the features to the embeddings directly (src/model.py:497-498 requires width == n_embd).
    # Otherwise a build-side Conv1D projection per modality maps feat_dim -> n_embd first (config 5:
    # 768-d BLIP / wav2vec2 features into the 1024-d GPT-2-medium stream).  The
    # projection has no reference counterpart: its parity is against this restatement only.
    feat_dim: Optional[int] = None

    @property
    def inner(self) -> int:
        return self.n_inner if self.n_inner is not None else 4 * self.n_embd

    @property
    def projected(self) -> bool:
        return self.feat_dim is not None and self.feat_dim != self.n_embd


def param_shapes(cfg: OracleConfig) -> Dict[str, tuple]:
    """Reference state_dict keys and shapes (src/model.py:94-99,257-258,276-284,387-392,605,608)."""
    E, V, P, F_ = cfg.n_embd, cfg.vocab_size, cfg.n_positions, cfg.inner
    s: Dict[str, tuple] = {
        "transformer.wte.weight": (V, E),
        "transformer.wpe.weight": (P, E),
    }
    for i in range(cfg.n_layer):
        p = f"transformer.h.{i}."
        s[p + "ln_1.weight"] = (E,)
        s[p + "ln_1.bias"] = (E,)
        s[p + "attn.c_attn.weight"] = (E, 3 * E)
        s[p + "attn.c_attn.bias"] = (3 * E,)
        s[p + "attn.c_proj.weight"] = (E, E)
        s[p + "attn.c_proj.bias"] = (E,)
        s[p + "ln_2.weight"] = (E,)
        s[p + "ln_2.bias"] = (E,)
        s[p + "crossattention.c_attn.weight"] = (E, 2 * E)
        s[p + "crossattention.c_attn.bias"] = (2 * E,)
        s[p + "crossattention.q_attn.weight"] = (E, E)
        s[p + "crossattention.q_attn.bias"] = (E,)
        s[p + "crossattention.c_proj.weight"] = (E, E)
        s[p + "crossattention.c_proj.bias"] = (E,)
        s[p + "ln_cross_attn.weight"] = (E,)
        s[p + "ln_cross_attn.bias"] = (E,)
        s[p + "mlp.c_fc.weight"] = (E, F_)
        s[p + "mlp.c_fc.bias"] = (F_,)
        s[p + "mlp.c_proj.weight"] = (F_, E)
        s[p + "mlp.c_proj.bias"] = (E,)
    s["transformer.ln_f.weight"] = (E,)
    s["transformer.ln_f.bias"] = (E,)
    s["emotion_head.weight"] = (NUM_EMOTIONS, E)
    if cfg.projected:  # build-side feature projections (not in the reference state_dict)
        for m in ("visual_proj", "audio_proj"):
            s[f"transformer.{m}.weight"] = (cfg.feat_dim, E)
            s[f"transformer.{m}.bias"] = (E,)
    return s


def init_params(cfg: OracleConfig, seed: int, perturb: bool = True) -> Dict[str, torch.Tensor]:
    """Seeded weights in reference layout (init rule of ``_init_weights`` src/model.py:359-375).

    Matrices ~ N(0, 0.02); every ``c_proj.weight`` ~ N(0, 0.02/sqrt(2L)) (:373-375).  With
    ``perturb`` the LayerNorm gains/shifts and biases get small random values instead of 1/0 so that
    parity exercises their gradients too (the reference accepts any state_dict).
    """
    g = torch.Generator().manual_seed(seed)
    out: Dict[str, torch.Tensor] = {}
    std = cfg.initializer_range
    for name, shape in param_shapes(cfg).items():
        if name.endswith("c_proj.weight"):
            t = torch.randn(shape, generator=g) * (std / math.sqrt(2 * cfg.n_layer))
        elif len(shape) == 2:
            t = torch.randn(shape, generator=g) * std
        elif ".ln_" in name or "ln_f" in name:
            if name.endswith("weight"):
                t = 1.0 + (0.1 * torch.randn(shape, generator=g) if perturb else torch.zeros(shape))
            else:
                t = 0.1 * torch.randn(shape, generator=g) if perturb else torch.zeros(shape)
        else:  # Conv1D bias
            t = 0.02 * torch.randn(shape, generator=g) if perturb else torch.zeros(shape)
        out[name] = t.float().contiguous()
    return out


def peak_cross_attention(P: Dict[str, torch.Tensor], n_layer: int, q_gain: float, kv_gain: float,
                         proj_gain: float) -> Dict[str, torch.Tensor]:
    """Scale every block's cross-attention query (``crossattention.q_attn.weight``), caption key/value
    (``crossattention.c_attn.weight``) and output (``crossattention.c_proj.weight``) projections in place.

    Under the N(0, 0.02) init the caption keys are raw ``wte`` rows through ``c_attn`` (src/model.py:219,460-463),
    so the cross-attention scores (src/model.py:150-152 via :211-222,311-329) are ~1e-3 and the softmax is flat:
    its query-side gradients are third-order small.  With gains of ~50 the scores reach O(1-5) (a peaked softmax,
    the trained-model regime) and the cross-attention gradients sit at the model's gradient scale.  Any
    state_dict is a valid reference input; the golden fixtures record the gains (``xpeak_gains``)."""
    for i in range(n_layer):
        p = f"transformer.h.{i}.crossattention."
        P[p + "q_attn.weight"] *= q_gain
        P[p + "c_attn.weight"] *= kv_gain
        P[p + "c_proj.weight"] *= proj_gain
    return P


def _conv1d(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """transformers ``Conv1D.forward``: ``addmm(bias, x.view(-1, in), W[in, out])``."""
    shp = x.shape[:-1] + (w.shape[1],)
    return torch.addmm(b, x.reshape(-1, x.shape[-1]), w).view(shp)


def _gelu_new(x: torch.Tensor) -> torch.Tensor:
    """transformers ``NewGELUActivation`` (ACT2FN['gelu_new'], used at src/model.py:259)."""
    return 0.5 * x * (1.0 + torch.tanh(math.sqrt(2.0 / math.pi) * (x + 0.044715 * torch.pow(x, 3.0))))


def _split_heads(t: torch.Tensor, H: int) -> torch.Tensor:  # src/model.py:190-193
    B, S, E = t.shape
    return t.view(B, S, H, E // H).permute(0, 2, 1, 3)


def _merge_heads(t: torch.Tensor) -> torch.Tensor:  # src/model.py:195-198
    B, H, S, d = t.shape
    return t.permute(0, 2, 1, 3).contiguous().view(B, S, H * d)


def _drop(x: torch.Tensor, keep: Optional[torch.Tensor], p: float) -> torch.Tensor:
    """``nn.Dropout`` in training mode with a given keep mask: x · keep · 1/(1-p) (torch scales the
    bernoulli noise by 1/(1-p) in the tensor's dtype).  keep None: identity (eval / p = 0)."""
    if keep is None or p == 0.0:
        return x
    return x * (keep.to(x.dtype) * torch.full([], 1.0 / (1.0 - p), dtype=torch.float32).to(x.dtype))


def _attn(q, k, v, causal: bool, mask_add: Optional[torch.Tensor] = None, keep: Optional[torch.Tensor] = None,
          p: float = 0.0) -> torch.Tensor:
    """``GPT2Attention._attn`` src/model.py:119-148 (scale_attn_weights=True, no layer-idx scaling;
    ``attn_dropout`` on the probabilities :142 with the given keep mask [B, H, Sq, Sk])."""
    w = torch.matmul(q, k.transpose(-1, -2))
    w = w / torch.full([], v.size(-1) ** 0.5, dtype=w.dtype)
    if causal:
        ql, kl = q.size(-2), k.size(-2)
        tril = torch.tril(torch.ones(kl, kl, dtype=torch.bool))[kl - ql: kl, :kl]
        w = torch.where(tril, w, torch.full([], torch.finfo(w.dtype).min, dtype=w.dtype))
    if mask_add is not None:
        w = w + mask_add
    w = F.softmax(w, dim=-1)
    w = _drop(w, keep, p)
    return torch.matmul(w, v)


def _layer_norm(x, P, name, eps):
    return F.layer_norm(x, (x.shape[-1],), P[name + ".weight"], P[name + ".bias"], eps)


def forward(P: Dict[str, torch.Tensor], cfg: OracleConfig, input_ids, token_type_ids=None,
            caption_ids=None, visual_feat=None, audio_feat=None, labels=None,
            emotion_labels=None, imgs=None, dropout=None) -> Dict[str, torch.Tensor]:
    """Fused model forward (``GPT2LMHeadModel.forward`` src/model.py:654-737).

    ``visual_feat`` is the pooled visual vector per sample: [B, E], or [B, Tv, E] (row 0 used,
    ``imgs[i][0]`` src/model.py:497).  ``imgs`` is the reference's own argument: ``imgs[i][0]`` is added
    to position 0, so a 2-D [B, E] ``imgs`` contributes the SCALAR imgs[i, 0] (broadcast) and a 3-D one
    its row 0.  ``audio_feat`` is ``auds`` [B, E] (:498).  ``caption_ids`` [B, S] is mandatory, as in
    the only runnable reference call.

    ``dropout`` = (attn_p, resid_p, embd_p, keep) replays training-mode dropout (src/model.py:142,245,
    266,506) with given keep masks: keep[site] bool, site numbers of include/ergm_hip.h (0 embeddings
    [B·S, E]; 3l+1..3l+3 the residual branches of block l [B·S, E]; 3L+1+2l / 3L+2+2l the attention /
    cross-attention probabilities of block l [B·H·S, Sk]).
    """
    if caption_ids is None:
        raise ValueError("caption_ids is required (src/model.py:521 reads caption_embeds unconditionally)")
    E, H, L, eps = cfg.n_embd, cfg.n_head, cfg.n_layer, cfg.layer_norm_epsilon
    wte, wpe = P["transformer.wte.weight"], P["transformer.wpe.weight"]
    B, S = input_ids.shape
    pa = pr = pe = 0.0
    keep = {}
    if dropout is not None:
        pa, pr, pe, keep = dropout

    def km(site, shape):  # keep mask of a site in the tensor's shape
        k = keep.get(site)
        return None if k is None else k.reshape(shape)
    if imgs is not None:
        if visual_feat is not None:
            raise ValueError("give imgs (reference semantics) or visual_feat, not both")
        visual_feat = imgs[:, :1].expand(B, imgs.shape[1]) if imgs.dim() == 2 else imgs
    inputs_embeds = F.embedding(input_ids, wte)                               # :459
    # :460-463 views captions as [-1, S] (caption length == S); [B, -1] is the same for Sc == S and
    # lets the KV-cache generation test score a response against fixed prompt captions (Sc != S)
    caption_embeds = F.embedding(caption_ids.view(B, -1), wte)
    enc_mask = torch.zeros(B, 1, 1, caption_embeds.shape[1])                  # :484-489 invert(ones)
    if visual_feat is not None:                                               # :495-498
        vis = visual_feat if visual_feat.dim() == 2 else visual_feat[:, 0]
        aud = audio_feat
        if cfg.projected:                                                     # build-side, config 5
            vis = _conv1d(vis, P["transformer.visual_proj.weight"], P["transformer.visual_proj.bias"])
            aud = _conv1d(aud, P["transformer.audio_proj.weight"], P["transformer.audio_proj.bias"])
        add = torch.zeros_like(inputs_embeds)
        add[:, 0] = vis
        add[:, 1] = aud
        inputs_embeds = inputs_embeds + add
    pos = F.embedding(torch.arange(S), wpe)                                   # :474-476,500
    h = inputs_embeds + pos                                                   # :501
    if token_type_ids is not None:
        h = h + F.embedding(token_type_ids, wte)                              # :502-504
    h = _drop(h, km(0, (B, S, E)), pe)                                        # :506
    Sc = caption_embeds.shape[1]
    for i in range(L):                                                        # :520-576
        p = f"transformer.h.{i}."
        r = h                                                                 # self-attn :297-309
        x = _layer_norm(h, P, p + "ln_1", eps)
        q, k, v = _conv1d(x, P[p + "attn.c_attn.weight"], P[p + "attn.c_attn.bias"]).split(E, dim=2)
        a = _attn(_split_heads(q, H), _split_heads(k, H), _split_heads(v, H), causal=True,
                  keep=km(3 * L + 1 + 2 * i, (B, H, S, S)), p=pa)
        a = _conv1d(_merge_heads(a), P[p + "attn.c_proj.weight"], P[p + "attn.c_proj.bias"])
        a = _drop(a, km(3 * i + 1, (B, S, E)), pr)                            # resid_dropout :245
        h = a + r
        r = h                                                                 # cross-attn :311-329
        x = _layer_norm(h, P, p + "ln_cross_attn", eps)
        q = _conv1d(x, P[p + "crossattention.q_attn.weight"], P[p + "crossattention.q_attn.bias"])
        k, v = _conv1d(caption_embeds, P[p + "crossattention.c_attn.weight"],
                       P[p + "crossattention.c_attn.bias"]).split(E, dim=2)
        a = _attn(_split_heads(q, H), _split_heads(k, H), _split_heads(v, H), causal=False,
                  mask_add=enc_mask, keep=km(3 * L + 2 + 2 * i, (B, H, S, Sc)), p=pa)
        a = _conv1d(_merge_heads(a), P[p + "crossattention.c_proj.weight"],
                    P[p + "crossattention.c_proj.bias"])
        a = _drop(a, km(3 * i + 2, (B, S, E)), pr)                            # resid_dropout :245
        h = r + a
        r = h                                                                 # MLP :331-334
        x = _layer_norm(h, P, p + "ln_2", eps)
        x = _conv1d(x, P[p + "mlp.c_fc.weight"], P[p + "mlp.c_fc.bias"])
        x = _gelu_new(x)
        x = _conv1d(x, P[p + "mlp.c_proj.weight"], P[p + "mlp.c_proj.bias"])
        x = _drop(x, km(3 * i + 3, (B, S, E)), pr)                            # mlp dropout :266
        h = r + x
    h = _layer_norm(h, P, "transformer.ln_f", eps)                            # :578
    logits = F.linear(h, wte)                                                 # :698 (tied)
    emo = F.linear(h[:, -1, :], P["emotion_head.weight"])                     # :700-701
    out = {"logits": logits, "emotion_logits": emo, "hidden": h}
    loss = None
    if labels is not None:                                                    # :704-718
        sl = logits[..., :-1, :].contiguous()
        lab = labels[..., 1:].contiguous()
        out["loss_lm"] = F.cross_entropy(sl.view(-1, sl.size(-1)), lab.view(-1), ignore_index=-100)
        loss = out["loss_lm"]
    if emotion_labels is not None:
        out["loss_emotion"] = F.cross_entropy(emo.view(-1, NUM_EMOTIONS), emotion_labels.view(-1))  # ignore -100
        loss = out["loss_emotion"] if loss is None else loss + out["loss_emotion"]
    out["loss"] = loss
    return out


def loss_and_grads(P: Dict[str, torch.Tensor], cfg: OracleConfig, batch: Dict[str, torch.Tensor], dropout=None):
    """Forward + ``loss.backward()`` (src/main.py:147-154); returns (outputs, grads by name)."""
    leaves = {k: v.detach().clone().requires_grad_(True) for k, v in P.items()}
    out = forward(leaves, cfg, **batch, dropout=dropout)
    out["loss"].backward()
    grads = {k: v.grad.detach().clone() if v.grad is not None else torch.zeros_like(v)
             for k, v in leaves.items()}
    return {k: (v.detach() if torch.is_tensor(v) else v) for k, v in out.items()}, grads


@dataclass
class AdamWState:
    step: int = 0
    exp_avg: Dict[str, torch.Tensor] = field(default_factory=dict)
    exp_avg_sq: Dict[str, torch.Tensor] = field(default_factory=dict)


def adamw_step(P: Dict[str, torch.Tensor], G: Dict[str, torch.Tensor], st: AdamWState, lr: float,
               betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.01) -> None:
    """torch.optim.AdamW single-tensor update (``torch.optim.AdamW(model.parameters(), lr)``,
    src/main.py:68): decoupled decay, lerp first moment, bias corrections in double precision."""
    b1, b2 = betas
    st.step += 1
    bc1 = 1 - b1 ** st.step
    bc2 = 1 - b2 ** st.step
    step_size = lr / bc1
    bc2_sqrt = math.sqrt(bc2)
    for k, p in P.items():
        g = G[k]
        m = st.exp_avg.setdefault(k, torch.zeros_like(p))
        v = st.exp_avg_sq.setdefault(k, torch.zeros_like(p))
        p.mul_(1 - lr * weight_decay)
        m.lerp_(g, 1 - b1)
        v.mul_(b2).addcmul_(g, g, value=1 - b2)
        denom = (v.sqrt() / bc2_sqrt).add_(eps)
        p.addcdiv_(m, denom, value=-step_size)


def poly_decay_lr(step: int, lr_init: float, num_warmup_steps: int, num_training_steps: int,
                  lr_end: float = 1e-7, power: float = 2.0) -> float:
    """LR after ``step`` scheduler steps: transformers ``get_polynomial_decay_schedule_with_warmup``
    (power=2 at src/main.py:93-95), restated from its published lambda."""
    if step < num_warmup_steps:
        mult = float(step) / float(max(1, num_warmup_steps))
    elif step > num_training_steps:
        mult = lr_end / lr_init
    else:
        lr_range = lr_init - lr_end
        decay_steps = num_training_steps - num_warmup_steps
        pct_remaining = 1 - (step - num_warmup_steps) / decay_steps
        mult = (lr_range * pct_remaining ** power + lr_end) / lr_init
    return lr_init * mult
