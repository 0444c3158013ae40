"""KV-cache generation (ergm_amd.generate) against the oracle's full-sequence forward: prefill logits
and every teacher-forced decode step's logits match a recompute over the whole prefix (captions fixed
to the prompt's), within the bf16 logits gate; nucleus sampling is seeded-deterministic and stops."""
import pytest
import torch

from ergm_amd.config import ERGMConfig, NO_DROPOUT
from ergm_amd.generate import KVCacheGenerator
from ergm_amd.model import GPT2LMHeadModel
from oracle import gpt2_oracle as O

pytestmark = pytest.mark.gpu
V, E, LYR, H, P = 500, 128, 2, 2, 64
LOGIT_ATOL = 0.06


def _setup(gpu, feat_dim=None):
    ocfg = O.OracleConfig(vocab_size=V, n_embd=E, n_layer=LYR, n_head=H, n_positions=P, feat_dim=feat_dim)
    P0 = O.init_params(ocfg, seed=11)
    model = GPT2LMHeadModel(ERGMConfig(vocab_size=V, n_embd=E, n_layer=LYR, n_head=H, n_positions=P,
                                       feat_dim=feat_dim, **NO_DROPOUT), device=gpu)
    model.load_state_dict(P0, strict=True)
    return ocfg, P0, model


@pytest.mark.parametrize("feat_dim", [None, 64])
def test_decode_steps_match_full_recompute(gpu, feat_dim):
    """feat_dim=64: the config-5 projections of the prompt's visual / audio vectors (E=128)."""
    ocfg, P0, model = _setup(gpu, feat_dim)
    Fd = feat_dim or E
    g = torch.Generator().manual_seed(4)
    S0 = 12
    ids = torch.randint(0, 490, (1, S0), generator=g)
    tt = torch.full((1, S0), 498)
    tt[:, 6:] = 499
    cap = torch.randint(0, 490, (1, S0), generator=g)
    vis, aud = 0.1 * torch.randn(1, Fd, generator=g), 0.1 * torch.randn(1, Fd, generator=g)
    gen = KVCacheGenerator(model, max_len=32)
    logits = gen.prefill(ids.to(gpu), tt.to(gpu), cap.to(gpu), vis.to(gpu), aud.to(gpu))
    forced = torch.randint(0, 490, (6,), generator=g)
    seq, types = ids, tt
    for t in range(len(forced) + 1):
        ref = O.forward(P0, ocfg, input_ids=seq, token_type_ids=types, caption_ids=cap, visual_feat=vis,
                        audio_feat=aud)["logits"][0, -1]
        assert (logits.float().cpu() - ref).abs().max().item() <= LOGIT_ATOL, t
        if t == len(forced):
            break
        tok = forced[t].view(1, 1)
        seq = torch.cat([seq, tok], 1)
        types = torch.cat([types, torch.full((1, 1), 499)], 1)
        logits = gen.step(tok.to(gpu), torch.full((1, 1), 499, device=gpu))


def test_nucleus_sampling_deterministic_and_bounded(gpu):
    _, _, model = _setup(gpu)
    ids = torch.randint(0, 490, (1, 10), generator=torch.Generator().manual_seed(1)).to(gpu)
    tt = torch.full((1, 10), 498, device=gpu)
    runs = []
    for _ in range(2):
        gen = KVCacheGenerator(model, max_len=24)
        gs = torch.Generator(device=gpu).manual_seed(7)
        runs.append(gen.nucleus_sampling(ids, tt, ids, top_p=0.9, eos_id=497, sp2_id=499, generator=gs))
    assert runs[0] == runs[1] and 1 <= len(runs[0]) <= 14
    assert all(0 <= t < V for t in runs[0])
