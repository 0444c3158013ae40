"""Response generation with a KV cache: ``nucleus_sampling`` of the reference trainer
(src/main.py:253-282) without its full-sequence recompute per token.

The reference re-runs the whole model on the growing sequence for every new token (and cannot run as
written: it passes no ``caption_ids``).  Here the prompt is encoded once (prefill, the
same kernels as training: causal attention over the prompt, cross-attention over the caption
embeddings), the per-layer self-attention keys/values are kept in a cache in HBM, the caption K/V of
every layer are computed once, and each new token costs one position through the stack: a row of
every GEMM, attention of one query over the cached keys (``ergm_attn_fwd`` with Sq = 1, non-causal —
all cached positions precede it), and the tied LM head for that row only.

The captions stay fixed while the response grows (the reference would need caption length == the
current sequence length, src/model.py:461, which generation cannot satisfy); the prompt's visual /
audio vectors enter at positions 0 and 1 as in training.  Batch 1, like the reference's test loop
(src/main.py:305-313).  Every op is a C-ABI kernel call; the sampling itself (softmax, sort, top-p
cut, multinomial over one [V] row) uses the reference's own torch calls on the device.
"""
from __future__ import annotations

from typing import List, Optional

import torch
import torch.nn.functional as F

from . import _lib as L
from . import ops


class KVCacheGenerator:
    def __init__(self, model, max_len: int = 1024):
        cfg = model.config
        if max_len > cfg.n_positions:
            raise ValueError(f"max_len {max_len} > n_positions {cfg.n_positions}")
        self.m, self.cfg = model, cfg
        self.E, self.H, self.L, self.F = cfg.n_embd, cfg.n_head, cfg.n_layer, cfg.inner
        self.max_len = max_len
        dev = model.flat.device
        self.dev = dev
        # per layer: self-attention K | V of every position so far, [max_len, 2E] bf16
        self.kv = [torch.empty(max_len, 2 * self.E, dtype=torch.bfloat16, device=dev) for _ in range(self.L)]
        self.xkv: List[torch.Tensor] = []
        self.n = 0

    # parameter views: fp32 master (biases, LayerNorm) and the bf16 shadow the GEMMs read
    def _f(self, name):
        return self.m.view(name)

    def _b(self, name):
        return self.m.view(name, self.m.flat_b16)

    def _ln(self, x, name):
        y, _, _ = ops.layernorm_fwd(x, self._f(name + ".weight"), self._f(name + ".bias"), self.cfg.layer_norm_epsilon)
        return y

    def _block(self, l: int, h: torch.Tensor, p0: int) -> None:
        """Rows h [n, E] (positions p0 .. p0+n-1) through block l, in place."""
        E, H, F_ = self.E, self.H, self.F
        n = h.shape[0]
        p = f"transformer.h.{l}."
        x = self._ln(h, p + "ln_1")
        qkv = ops.gemm(x, self._b(p + "attn.c_attn.weight"), n, 3 * E, E, L.MK, L.KN, out_dtype=torch.bfloat16,
                       epilogue=L.EPI_BIAS, bias=self._f(p + "attn.c_attn.bias"))
        cache = self.kv[l]
        cache[p0:p0 + n].copy_(qkv[:, E:])
        k, v = cache[:, :E], cache[:, E:]
        if p0 == 0:   # prefill: causal over the prompt
            a, _ = ops.attn_fwd(qkv[:, :E], k, v, 1, H, n, n, True)
        else:         # one new position: every cached key precedes it
            a, _ = ops.attn_fwd(qkv[:, :E], k, v, 1, H, n, p0 + n, False)
        ops.gemm(a, self._b(p + "attn.c_proj.weight"), n, E, E, L.MK, L.KN, out=h, epilogue=L.EPI_BIAS_RESID,
                 bias=self._f(p + "attn.c_proj.bias"), aux=h)
        x = self._ln(h, p + "ln_cross_attn")
        q = ops.gemm(x, self._b(p + "crossattention.q_attn.weight"), n, E, E, L.MK, L.KN, out_dtype=torch.bfloat16,
                     epilogue=L.EPI_BIAS, bias=self._f(p + "crossattention.q_attn.bias"))
        xkv = self.xkv[l]
        a, _ = ops.attn_fwd(q, xkv[:, :E], xkv[:, E:], 1, H, n, xkv.shape[0], False)
        ops.gemm(a, self._b(p + "crossattention.c_proj.weight"), n, E, E, L.MK, L.KN, out=h,
                 epilogue=L.EPI_BIAS_RESID, bias=self._f(p + "crossattention.c_proj.bias"), aux=h)
        x = self._ln(h, p + "ln_2")
        pre = torch.empty(n, F_, dtype=torch.bfloat16, device=self.dev)
        act = ops.gemm(x, self._b(p + "mlp.c_fc.weight"), n, F_, E, L.MK, L.KN, out_dtype=torch.bfloat16,
                       epilogue=L.EPI_BIAS_GELU, bias=self._f(p + "mlp.c_fc.bias"), aux_out=pre)
        ops.gemm(act, self._b(p + "mlp.c_proj.weight"), n, E, F_, L.MK, L.KN, out=h, epilogue=L.EPI_BIAS_RESID,
                 bias=self._f(p + "mlp.c_proj.bias"), aux=h)

    def _head(self, h_last: torch.Tensor) -> torch.Tensor:
        x = self._ln(h_last, "transformer.ln_f")
        lay = self.m.layout
        logits = ops.gemm(x, self._b("__wte_pad"), 1, lay.vocab_pad, self.E, L.MK, L.NK, out_dtype=torch.float32)
        return logits[0, :lay.vocab]

    @torch.no_grad()
    def prefill(self, input_ids, token_type_ids, caption_ids, imgs=None, auds=None) -> torch.Tensor:
        """Encode the prompt [1, S0]; returns the next-token logits [V] (fp32)."""
        self.m.refresh_bf16()
        if input_ids.dim() != 2 or input_ids.shape[0] != 1:
            raise ValueError("generation runs one sequence at a time (batch 1)")
        S0 = input_ids.shape[1]
        if S0 >= self.max_len:
            raise ValueError("prompt longer than max_len")
        wte, wpe = self._f("__wte_pad"), self._f("transformer.wpe.weight")
        Fd = self.m.layout.Fd
        vis = None if imgs is None else imgs.float().reshape(1, -1, Fd)[:, 0]
        aud = None if auds is None else auds.float().reshape(1, Fd)
        if vis is not None and Fd != self.E:  # config 5: the build-side projections (Conv1D), MFMA GEMMs
            vis, aud = (ops.gemm(x.to(torch.bfloat16), self._b(f"transformer.{m}.weight"), 1, self.E, Fd, L.MK, L.KN,
                                 out_dtype=torch.float32, epilogue=L.EPI_BIAS, bias=self._f(f"transformer.{m}.bias"))
                        for x, m in ((vis, "visual_proj"), (aud, "audio_proj")))
        h, _ = ops.embed_fwd(input_ids, token_type_ids, input_ids, wte, wpe, vis, aud)
        _, cap = ops.embed_fwd(caption_ids, None, caption_ids, wte, wpe)
        Sc = caption_ids.shape[1]
        self.xkv = [ops.gemm(cap, self._b(f"transformer.h.{l}.crossattention.c_attn.weight"), Sc, 2 * self.E,
                             self.E, L.MK, L.KN, out_dtype=torch.bfloat16, epilogue=L.EPI_BIAS,
                             bias=self._f(f"transformer.h.{l}.crossattention.c_attn.bias")) for l in range(self.L)]
        for l in range(self.L):
            self._block(l, h, 0)
        self.n = S0
        return self._head(h[S0 - 1:S0])

    @torch.no_grad()
    def step(self, token: torch.Tensor, token_type: torch.Tensor) -> torch.Tensor:
        """Append one token (ids [1, 1]) at position n; returns the logits [V] for position n + 1."""
        if self.n >= self.max_len:
            raise ValueError("KV cache full")
        wte, wpe = self._f("__wte_pad"), self._f("transformer.wpe.weight")
        h, _ = ops.embed_fwd(token, token_type, token, wte, wpe[self.n:])  # wpe row n is position 0 of the view
        for l in range(self.L):
            self._block(l, h, self.n)
        self.n += 1
        return self._head(h)

    @torch.no_grad()
    def nucleus_sampling(self, input_ids, token_type_ids, caption_ids, top_p: float, eos_id: int, sp2_id: int,
                         imgs=None, auds=None, generator: Optional[torch.Generator] = None) -> List[int]:
        """src/main.py:253-282: sample until eos or max_len, the response typed as speaker 2."""
        logits = self.prefill(input_ids, token_type_ids, caption_ids, imgs, auds)
        out: List[int] = []
        tt = torch.full((1, 1), sp2_id, dtype=torch.long, device=self.dev)
        for pos in range(input_ids.shape[1], self.max_len):
            probs = F.softmax(logits.unsqueeze(0), dim=-1)
            sorted_probs, sorted_idxs = torch.sort(probs, descending=True)
            cum = torch.cumsum(sorted_probs, dim=-1)
            remove = cum > top_p
            remove[:, 1:] = remove[:, :-1].clone()
            remove[:, 0] = False
            sorted_probs[remove] = 0.0
            sorted_probs /= torch.sum(sorted_probs, dim=-1, keepdim=True)
            probs = torch.zeros_like(probs).scatter_(-1, sorted_idxs, sorted_probs)
            idx = torch.multinomial(probs, 1, generator=generator)
            tok = int(idx.item())
            out.append(tok)
            if tok == eos_id or pos + 1 >= self.max_len:
                break
            logits = self.step(idx.view(1, 1), tt)
        return out
