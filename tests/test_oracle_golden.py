"""The CPU oracle against the golden fixtures captured from the reference (tests/golden/make_golden.py).

These pin the oracle everywhere (including the GPU box, where /root/reference does not exist); the
HIP path is then checked against the oracle in the gpu tests.
"""
import os

import numpy as np
import pytest
import torch

from oracle import gpt2_oracle as O

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _load(name):
    z = np.load(os.path.join(GOLD, name))
    return {k: z[k] for k in z.files}


def _batch(rec):
    b = {}
    for k, v in rec.items():
        if k.startswith("in_"):
            b[k[3:]] = torch.from_numpy(v)
    return b


def _cfg(rec):
    V, E, Lyr, H, P = (int(x) for x in rec["config"])
    return O.OracleConfig(vocab_size=V, n_embd=E, n_layer=Lyr, n_head=H, n_positions=P)


def _params(rec, cfg):
    """The fixture's weights: the oracle's seeded init, with the peaked cross-attention gains when recorded."""
    P = O.init_params(cfg, seed=int(rec["seed"]))
    if "xpeak_gains" in rec:
        O.peak_cross_attention(P, cfg.n_layer, *(float(x) for x in rec["xpeak_gains"]))
    return P


def _rel(a, b):
    a, b = torch.as_tensor(a).double(), torch.as_tensor(b).double()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize("name", ["tiny_e64.npz", "small_e128_v500.npz", "xpeak_e128.npz"])
def test_oracle_matches_reference_small(name):
    rec = _load(name)
    cfg = _cfg(rec)
    P = _params(rec, cfg)
    out, grads = O.loss_and_grads(P, cfg, _batch(rec))
    assert abs(out["loss"].item() - float(rec["loss"])) <= 1e-5 * abs(float(rec["loss"]))
    assert _rel(out["emotion_logits"], rec["emotion_logits"]) < 1e-5
    assert _rel(out["logits"], rec["logits"]) < 1e-5
    for k, g in grads.items():
        if "grad:" + k in rec:
            assert _rel(g, rec["grad:" + k]) < 1e-4, k
        else:
            ref = float(rec["gradnorm:" + k])
            assert abs(g.double().norm().item() - ref) <= 1e-4 * max(ref, 1e-12), k
            assert _rel(g.reshape(-1)[:32], rec["gradhead:" + k]) < 1e-3, k


@pytest.mark.parametrize("name", ["c1_gpt2small_textonly.npz", "c2slice_gpt2small_fusion.npz", "xpeak_c2slice.npz"])
def test_oracle_matches_reference_gpt2_small(name):
    rec = _load(name)
    cfg = _cfg(rec)
    P = _params(rec, cfg)
    out, grads = O.loss_and_grads(P, cfg, _batch(rec))
    assert abs(out["loss"].item() - float(rec["loss"])) <= 1e-5 * abs(float(rec["loss"]))
    assert _rel(out["emotion_logits"], rec["emotion_logits"]) < 1e-5
    assert _rel(out["logits"][:, :4, :64], rec["logits_head"]) < 1e-5
    assert _rel(out["logits"][:, -2:, -64:], rec["logits_tail"]) < 1e-5
    for k, g in grads.items():
        ref = float(rec["gradnorm:" + k])
        assert abs(g.double().norm().item() - ref) <= 1e-4 * max(ref, 1e-12), k


def test_adamw_and_schedule_restatement():
    rec = _load("adamw_sched.npz")
    keys = sorted({k.split(":", 1)[1] for k in rec if k.startswith("p0:")})
    P = {k: torch.from_numpy(rec["p0:" + k]).clone() for k in keys}
    st = O.AdamWState()
    for i in range(3):
        G = {k: torch.from_numpy(rec[f"g{i}:" + k]) for k in keys}
        lr = O.poly_decay_lr(i, 2e-5, 1, 5)
        assert lr == pytest.approx(float(rec["lrs"][i]), rel=1e-12, abs=0)
        O.adamw_step(P, G, st, lr)
    for k in keys:
        np.testing.assert_allclose(P[k].numpy(), rec["p3:" + k], rtol=1e-6, atol=1e-9)
    lr0, warm, total = rec["sched_args"]
    for step, want in enumerate(rec["sched_lrs"]):
        assert O.poly_decay_lr(step, float(lr0), int(warm), int(total)) == pytest.approx(float(want), rel=1e-9)
