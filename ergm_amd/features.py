"""On-GPU pooling of the encoder outputs that become ERGM's visual / audio vectors.

The reference featurises offline (data_process/feature_extraction.py): wav2vec2-base-960h
``last_hidden_state`` [1, T_audio, 768] and BLIP-vision ``last_hidden_state`` [1, 197, 768] for each
keyframe, each mean-pooled over its frames/patches (``torch.mean(features, dim=1)``, :63 and :69) into
the 768-d vectors the dataset stores and the model adds at positions 0 and 1 (src/model.py:495-498).
The encoders themselves download from the network and are out of scope; this module does the pooling
on the GPU (one HIP kernel, ``ergm_feat_pool``) for a whole batch, with per-sample valid lengths for
padded audio, so encoder outputs already in HBM feed the model (and at config 5 its projection GEMMs)
without a host round trip.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from . import ops


def mean_pool(hidden: torch.Tensor, lengths: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``torch.mean(hidden, dim=1)`` (feature_extraction.py:63,69) over the first ``lengths[b]`` frames
    of each sample; [B, T, D] f32/bf16 -> [B, D] f32."""
    return ops.feat_pool(hidden, lengths)


def pool_encoder_outputs(image_hidden: torch.Tensor, audio_hidden: torch.Tensor,
                         audio_lengths: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """(visual_feat [B, D], audio_feat [B, D]) from BLIP-vision [B, 197, D] and wav2vec2 [B, T, D] outputs."""
    return mean_pool(image_hidden), mean_pool(audio_hidden, audio_lengths)
