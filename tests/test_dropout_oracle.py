"""CPU checks of the dropout checker (oracle/philox.py) and of the oracle's mask replay.

The keep masks are the build's (include/ergm_hip.h ergm_dropout: Philox4x32-10 of (seed, forward
number, site, element)); the reference's own masks come from torch's generator inside nn.Dropout
(src/model.py:142,245,266,506) and are not reproducible, so parity replays the build's masks through
the oracle.  Here: the restated Philox against the Random123 known-answer vectors, the mask's keep
rate / independence, and that the oracle's replay is nn.Dropout's arithmetic."""
import numpy as np
import torch

from oracle import gpt2_oracle as O
from oracle import philox as X


def test_philox_known_answers():
    for ctr, key, want in X.KAT:
        got = X.philox4x32_10(*[np.uint32(c) for c in ctr], *key)
        assert [int(v) for v in got] == list(want)


def test_keep_rate_and_independence():
    p = 0.1
    m = X.keep_mask(seed=2024, offset=1, site=5, p=p, rows=512, cols=768)
    n = m.size
    sigma = (p * (1 - p) / n) ** 0.5
    assert abs((1 - m.mean()) - p) < 5 * sigma
    other_site = X.keep_mask(2024, 1, 6, p, 512, 768)
    other_step = X.keep_mask(2024, 2, 5, p, 512, 768)
    other_seed = X.keep_mask(2025, 1, 5, p, 512, 768)
    for o in (other_site, other_step, other_seed):
        agree = (o == m).mean()  # independent masks agree on p² + (1-p)² of the elements
        assert abs(agree - (p * p + (1 - p) ** 2)) < 0.01
    # a pure function, and rows offset by row0 are the same global rows
    assert np.array_equal(m, X.keep_mask(2024, 1, 5, p, 512, 768))
    assert np.array_equal(m[100:164], X.keep_mask(2024, 1, 5, p, 64, 768, row0=100))
    assert X.keep_mask(1, 1, 1, 0.0, 4, 8).all()


def test_oracle_dropout_replay_is_nn_dropout():
    """With all-keep masks the replay is the identity; with a mask it is x·keep/(1-p) at the
    reference's positions (embeddings, probabilities, residual branches), so the loss changes."""
    from ergm_amd.data import synthetic_batch
    cfg = O.OracleConfig(vocab_size=256, n_embd=64, n_layer=2, n_head=1, n_positions=64)
    P = O.init_params(cfg, seed=3)
    b = synthetic_batch(2, 16, n_turns=2, feat_dim=64, seed=4, vocab_hi=250, sp1=254, sp2=255, eos=249)
    base = O.forward(P, cfg, **b)["loss"]
    L, T, H, S, E = 2, 32, 1, 16, 64
    ones = {0: torch.ones(T, E, dtype=torch.bool)}
    for l in range(L):
        for k in range(3):
            ones[3 * l + 1 + k] = torch.ones(T, E, dtype=torch.bool)
        ones[3 * L + 1 + 2 * l] = torch.ones(2 * H * S, S, dtype=torch.bool)
        ones[3 * L + 2 + 2 * l] = torch.ones(2 * H * S, S, dtype=torch.bool)
    same = O.forward(P, cfg, **b, dropout=(0.0, 0.0, 0.0, ones))["loss"]
    assert torch.equal(base, same)
    keep = {s: torch.from_numpy(X.keep_mask(7, 1, s, 0.1, v.shape[0], v.shape[1])) for s, v in ones.items()}
    dropped = O.forward(P, cfg, **b, dropout=(0.1, 0.1, 0.1, keep))["loss"]
    assert torch.isfinite(dropped) and abs(dropped.item() - base.item()) > 1e-4
    # the embedding site alone: h0 = drop(emb) exactly (nn.functional.dropout's arithmetic with this mask)
    only = {0: keep[0]}
    h_ref = O.forward(P, cfg, **b, dropout=(0.0, 0.0, 0.1, only))
    assert torch.isfinite(h_ref["loss"])
