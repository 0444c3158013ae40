"""Flat parameter layout of the fused model, and the reference state_dict names as views into it.

All parameters live in ONE fp32 buffer (plus a bf16 shadow with identical offsets that the GEMMs
read, and one fp32 gradient buffer with the same layout).  The order is the order in which the
backward pass finishes each tensor's gradient, so data-parallel all-reduce buckets are contiguous
ranges that become ready one after another:

    emotion_head | ln_f | block L-1 | ... | block 0 | stacked caption K/V proj (all blocks) | wpe
    | [visual_proj | audio_proj] | wte

The tied ``wte``/``lm_head`` weight is padded to a multiple of 64 rows with zero rows (zero logits,
zero gradients, AdamW keeps them 0) so the LM-head GEMMs need no N/K tail handling.  The
cross-attention ``c_attn`` weights of all blocks are stored stacked as one [E, L·2E] matrix (the
caption K/V projections of every block run as one GEMM); per-block names are strided views.

When the pooled audio / visual features are narrower than the backbone (config 5: 768-d features,
n_embd 1024) the layout also holds the build-side feature projections ``transformer.visual_proj`` /
``transformer.audio_proj`` (Conv1D [Fd, E] + bias, bias right after its weight); the reference has no
such tensors (it adds 768-d features to a 768-d stream, src/model.py:497-498).

Names follow the reference state_dict (src/model.py:94-99,257-258,276-284,387-392,605,608).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Tuple

from ._lib import LAYER_TENSORS

ALIGN = 64  # elements (256 B of fp32, 128 B of bf16)


def _al(x: int) -> int:
    return (x + ALIGN - 1) // ALIGN * ALIGN


@dataclass
class View:
    offset: int            # element offset of element [0, 0] in the flat buffer
    shape: Tuple[int, ...]
    stride: Tuple[int, ...]

    @property
    def numel(self) -> int:
        n = 1
        for s in self.shape:
            n *= s
        return n


@dataclass
class Layout:
    vocab: int
    vocab_pad: int
    E: int
    L: int
    F: int
    P: int
    Fd: int                   # pooled feature width (== E: no projection)
    total: int
    views: Dict[str, View]
    layer_base: List[int]     # element offset of block i's tensor group
    layer_stride: int         # layer_base[i+1] - layer_base[i] (negative: blocks stored in reverse)
    layer_off: List[int]      # offsets of the 18 per-block tensors inside a block group
    seg: Dict[str, Tuple[int, int]]   # named contiguous segments [start, end)

    def layer_names(self, i: int) -> List[str]:
        return [f"transformer.h.{i}." + t for t in LAYER_TENSORS]


def build_layout(vocab: int, E: int, L: int, F: int, P: int, num_emotions: int = 7, feat_dim=None) -> Layout:
    Fd = E if not feat_dim else feat_dim
    vocab_pad = _al(vocab)
    views: Dict[str, View] = {}
    seg: Dict[str, Tuple[int, int]] = {}
    off = 0

    def put(name, shape):
        nonlocal off
        n = 1
        for s in shape:
            n *= s
        stride = (shape[1], 1) if len(shape) == 2 else (1,)
        views[name] = View(off, tuple(shape), stride)
        off = _al(off + n)

    s0 = off
    put("emotion_head.weight", (num_emotions, E))
    put("transformer.ln_f.weight", (E,))
    put("transformer.ln_f.bias", (E,))
    seg["head"] = (s0, off)
    shapes = {"ln_1.weight": (E,), "ln_1.bias": (E,), "attn.c_attn.weight": (E, 3 * E), "attn.c_attn.bias": (3 * E,),
              "attn.c_proj.weight": (E, E), "attn.c_proj.bias": (E,), "ln_cross_attn.weight": (E,),
              "ln_cross_attn.bias": (E,), "crossattention.q_attn.weight": (E, E),
              "crossattention.q_attn.bias": (E,), "crossattention.c_proj.weight": (E, E),
              "crossattention.c_proj.bias": (E,), "ln_2.weight": (E,), "ln_2.bias": (E,),
              "mlp.c_fc.weight": (E, F), "mlp.c_fc.bias": (F,), "mlp.c_proj.weight": (F, E), "mlp.c_proj.bias": (E,)}
    layer_base = [0] * L
    for i in reversed(range(L)):
        b = off
        layer_base[i] = b
        for t in LAYER_TENSORS:
            put(f"transformer.h.{i}." + t, shapes[t])
        seg[f"layer{i}"] = (b, off)
    layer_off = [views["transformer.h.0." + t].offset - layer_base[0] for t in LAYER_TENSORS]
    layer_stride = (layer_base[1] - layer_base[0]) if L > 1 else 0
    s0 = off
    capw = off
    off = _al(off + E * L * 2 * E)
    capb = off
    off = _al(off + L * 2 * E)
    for i in range(L):
        views[f"transformer.h.{i}.crossattention.c_attn.weight"] = View(capw + i * 2 * E, (E, 2 * E), (L * 2 * E, 1))
        views[f"transformer.h.{i}.crossattention.c_attn.bias"] = View(capb + i * 2 * E, (2 * E,), (1,))
    views["__capkv_w"] = View(capw, (E, L * 2 * E), (L * 2 * E, 1))
    views["__capkv_b"] = View(capb, (L * 2 * E,), (1,))
    put("transformer.wpe.weight", (P, E))
    if Fd != E:
        for m in ("visual_proj", "audio_proj"):
            put(f"transformer.{m}.weight", (Fd, E))
            put(f"transformer.{m}.bias", (E,))
    seg["capwpe"] = (s0, off)
    wte_off = off
    views["transformer.wte.weight"] = View(wte_off, (vocab, E), (E, 1))
    views["__wte_pad"] = View(wte_off, (vocab_pad, E), (E, 1))
    off = _al(off + vocab_pad * E)
    seg["wte"] = (wte_off, off)
    seg["embed"] = (s0, off)
    return Layout(vocab, vocab_pad, E, L, F, P, Fd, off, views, layer_base, layer_stride, layer_off, seg)


def state_dict_names(layout: Layout) -> List[str]:
    """Reference state_dict key order (GPT2LMHeadModel with tied lm_head)."""
    names = ["transformer.wte.weight", "transformer.wpe.weight"]
    order = ["ln_1.weight", "ln_1.bias", "attn.c_attn.weight", "attn.c_attn.bias", "attn.c_proj.weight",
             "attn.c_proj.bias", "ln_2.weight", "ln_2.bias", "crossattention.c_attn.weight",
             "crossattention.c_attn.bias", "crossattention.q_attn.weight", "crossattention.q_attn.bias",
             "crossattention.c_proj.weight", "crossattention.c_proj.bias", "ln_cross_attn.weight",
             "ln_cross_attn.bias", "mlp.c_fc.weight", "mlp.c_fc.bias", "mlp.c_proj.weight", "mlp.c_proj.bias"]
    for i in range(layout.L):
        names += [f"transformer.h.{i}." + t for t in order]
    names += ["transformer.ln_f.weight", "transformer.ln_f.bias", "lm_head.weight", "emotion_head.weight"]
    if layout.Fd != layout.E:  # build-side feature projections (config 5)
        names += [f"transformer.{m}.{t}" for m in ("visual_proj", "audio_proj") for t in ("weight", "bias")]
    return names


def dp_buckets(layout: Layout) -> List[Tuple[int, int]]:
    """Contiguous gradient ranges in backward-completion order: (head + block L-1), block L-2, …,
    block 0, (caption K/V + wpe + wte).  Bucket k is ready after backward stage k."""
    L = layout.L
    b = [(layout.seg["head"][0], layout.seg[f"layer{L - 1}"][1])]
    for i in reversed(range(L - 1)):
        b.append(layout.seg[f"layer{i}"])
    b.append(layout.seg["embed"])
    return b


# Conv1D weight matrices the executor reads only through the bf16 shadow (ergm_model_params *_b)
_SHADOW_ONLY = ("attn.c_attn.weight", "attn.c_proj.weight", "crossattention.q_attn.weight",
                "crossattention.c_proj.weight", "mlp.c_fc.weight", "mlp.c_proj.weight")


def master_read_ranges(layout: Layout, fp8: bool = False) -> List[Tuple[int, int]]:
    """Sorted, merged [start, end) element ranges of the fp32 master that the executor reads directly
    (LayerNorm parameters, biases, wpe, the emotion head, the tied wte): everything except the Conv1D
    weight matrices, which it reads through the bf16 shadow (the fp8 weight quantiser too, so ``fp8``
    changes nothing).  The sharded optimizer update (dist.py, ZeRO-1) keeps these replicated in fp32 on
    every rank."""
    skip = {f"transformer.h.{i}.{t}" for i in range(layout.L) for t in _SHADOW_ONLY}
    skip |= {"transformer.visual_proj.weight", "transformer.audio_proj.weight", "transformer.wte.weight"}
    skip |= {f"transformer.h.{i}.crossattention.c_attn.{t}" for i in range(layout.L) for t in ("weight", "bias")}
    skip.add("__capkv_w")
    iv = sorted((v.offset, v.offset + v.numel) for k, v in layout.views.items() if k not in skip)
    out: List[Tuple[int, int]] = []
    for a, b in iv:
        if out and a <= out[-1][1]:
            out[-1] = (out[-1][0], max(out[-1][1], b))
        else:
            out.append((a, b))
    return out
