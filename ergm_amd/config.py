"""Model / run configuration mirroring the ``GPT2Config`` fields the reference path reads.

Reference: ``GPT2Config`` fields used by src/model.py (n_embd/n_head/n_layer/n_inner,
max_position_embeddings, layer_norm_epsilon, activation_function='gelu_new', dropouts,
scale_attn_weights) and the special-token layout of src/main.py:47-63 (vocab 50257 + bos/sp1/sp2).
"""
from __future__ import annotations

from dataclasses import dataclass, asdict
from typing import Optional

# Special tokens after ``tokenizer.add_special_tokens`` (src/main.py:47-58): GPT-2 BPE has
# 50257 entries with eos=50256; bos, sp1, sp2 are appended.
GPT2_BASE_VOCAB = 50257
EOS_ID = 50256
BOS_ID = 50257
SP1_ID = 50258
SP2_ID = 50259
VOCAB_SIZE = 50260
NUM_EMOTIONS = 7  # src/model.py:607


@dataclass
class ERGMConfig:
    vocab_size: int = VOCAB_SIZE
    n_embd: int = 768
    n_layer: int = 12
    n_head: int = 12
    n_positions: int = 1024
    n_inner: Optional[int] = None
    layer_norm_epsilon: float = 1e-5
    initializer_range: float = 0.02
    # dropout probabilities (GPT2Config defaults = the "gpt2" checkpoint the reference fine-tunes,
    # src/main.py:62): applied in train() mode; 0 gives the deterministic path the parity goldens use
    attn_pdrop: float = 0.1
    resid_pdrop: float = 0.1
    embd_pdrop: float = 0.1
    # width of the pooled audio / visual features (data_process/feature_extraction.py:63,69 → 768).
    # When it differs from n_embd a build-side projection GEMM maps it (config 5).
    feat_dim: Optional[int] = None
    # config 5: forward Conv1D GEMMs on fp8 (e4m3, per-row activation / per-column weight scales,
    # block-scaled MFMA at 2x the bf16 rate); LM head, backward and optimizer stay bf16 / fp32
    fp8: bool = False

    @property
    def inner(self) -> int:
        return self.n_inner if self.n_inner is not None else 4 * self.n_embd

    @property
    def head_dim(self) -> int:
        return self.n_embd // self.n_head

    def validate(self) -> None:
        if self.n_embd % self.n_head != 0:
            # same message family as src/model.py:81-85
            raise ValueError(f"`embed_dim` must be divisible by num_heads (got `embed_dim`: {self.n_embd} "
                             f"and `num_heads`: {self.n_head}).")
        for name in ("attn_pdrop", "resid_pdrop", "embd_pdrop"):
            p = getattr(self, name)
            if not 0.0 <= p < 1.0:
                raise ValueError(f"{name} must be in [0, 1) (got {p})")

    def to_dict(self):
        return asdict(self)


def gpt2_small(**kw) -> ERGMConfig:
    return ERGMConfig(n_embd=768, n_layer=12, n_head=12, **kw)


def gpt2_medium(**kw) -> ERGMConfig:
    return ERGMConfig(n_embd=1024, n_layer=24, n_head=16, **kw)


# the deterministic path (every dropout off): parity goldens / oracle comparisons without mask replay
NO_DROPOUT = dict(attn_pdrop=0.0, resid_pdrop=0.0, embd_pdrop=0.0)
