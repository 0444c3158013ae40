"""Optimizer-state interchange with the reference's checkpoints (src/main.py:68,107,188): the reference
optimizes ``torch.optim.AdamW(model.parameters())`` and saves its per-tensor state; FusedAdamW holds one
flat state.  Pinned by tests/golden/optim_ref.npz, written by running the reference model and optimizer
(tests/golden/make_golden.py --only optim): its parameter order, the state after two steps, the step-3
gradient, and the parameters / state after the third step.

CPU: the parameter order and the flat <-> per-tensor converters.  GPU: FusedAdamW resumes from the
reference state and takes the reference's third step; torch.optim.AdamW resumes from FusedAdamW's
reference-format state and takes the same step; the Trainer loads a reference-format checkpoint.
"""
import json
import os
import tempfile

import numpy as np
import pytest
import torch

from ergm_amd.optim import flat_from_reference, reference_from_flat, reference_param_names
from ergm_amd.params import build_layout

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "optim_ref.npz")


def _fixture():
    z = np.load(GOLD)
    rec = {k: z[k] for k in z.files}
    order = json.loads(bytes(rec["param_order_json"]).decode())
    group = json.loads(bytes(rec["group_json"]).decode())
    V, E, L, H, P = (int(x) for x in rec["config"])
    return rec, order, group, (V, E, L, H, P)


def _ref_state(rec, order, group, tag="st2"):
    """The reference optimizer's state_dict as torch.optim.AdamW.state_dict() returns it."""
    state = {i: {"step": torch.tensor(float(rec[f"st2:{n}:step"])),
                 "exp_avg": torch.from_numpy(rec[f"{tag}:{n}:exp_avg"]),
                 "exp_avg_sq": torch.from_numpy(rec[f"{tag}:{n}:exp_avg_sq"])} for i, n in enumerate(order)}
    g = dict(group)
    g["betas"] = tuple(g["betas"])
    g["params"] = list(range(len(order)))
    return {"state": state, "param_groups": [g]}


def test_reference_parameter_order_is_pinned():
    rec, order, group, (V, E, L, H, P) = _fixture()
    lay = build_layout(V, E, L, 4 * E, P)
    assert reference_param_names(lay) == order


def test_flat_reference_round_trip():
    rec, order, group, (V, E, L, H, P) = _fixture()
    lay = build_layout(V, E, L, 4 * E, P)
    sd = _ref_state(rec, order, group)
    like = torch.zeros(lay.total)
    m, v, step, hp = flat_from_reference(lay, sd, like)
    assert step == 2.0 and hp["lr"] == group["lr"] and hp["betas"] == (0.9, 0.999)
    # padding (wte rows past the vocabulary, alignment gaps) stays zero: the moments cover exactly the parameters
    n_param = sum(int(np.prod(rec[f"st2:{n}:exp_avg"].shape)) for n in order)
    assert int((m != 0).sum()) <= n_param and float(m.abs().sum()) > 0
    back = reference_from_flat(lay, m, v, torch.tensor(step), {"lr": hp["lr"], "betas": hp["betas"],
                                                                "eps": hp["eps"], "weight_decay": hp["weight_decay"],
                                                                "params": [None]})
    assert back["param_groups"][0]["params"] == list(range(len(order)))
    for i, n in enumerate(order):
        assert torch.equal(back["state"][i]["exp_avg"], sd["state"][i]["exp_avg"]), n
        assert torch.equal(back["state"][i]["exp_avg_sq"], sd["state"][i]["exp_avg_sq"]), n
        assert float(back["state"][i]["step"]) == 2.0
    # a reference state for another configuration is refused
    with pytest.raises(ValueError):
        flat_from_reference(build_layout(V, E, L + 1, 4 * E, P), sd, torch.zeros(build_layout(V, E, L + 1, 4 * E, P).total))
    # so are per-parameter steps that differ (one flat step cannot hold them)
    sd["state"][0] = dict(sd["state"][0], step=torch.tensor(1.0))
    with pytest.raises(ValueError):
        flat_from_reference(lay, sd, like)


def _model(gpu, rec, dims):
    from ergm_amd.config import ERGMConfig, NO_DROPOUT
    from ergm_amd.model import GPT2LMHeadModel
    V, E, L, H, P = dims
    model = GPT2LMHeadModel(ERGMConfig(vocab_size=V, n_embd=E, n_layer=L, n_head=H, n_positions=P, **NO_DROPOUT),
                            device=gpu)
    model.load_state_dict({k[3:]: torch.from_numpy(v) for k, v in rec.items() if k.startswith("p2:")}, strict=False)
    return model


@pytest.mark.gpu
def test_fused_adamw_resumes_reference_state_and_back(gpu):
    from ergm_amd.optim import FusedAdamW
    rec, order, group, dims = _fixture()
    model = _model(gpu, rec, dims)
    opt = FusedAdamW([model.flat], lr=1.0, model=model)  # lr comes from the loaded state
    opt.load_state_dict(_ref_state(rec, order, group))
    assert opt.param_groups[0]["lr"] == group["lr"]
    g = torch.zeros_like(model.flat)
    for n in order:
        model.view(n, g).copy_(torch.from_numpy(rec[f"g3:{n}"]))
    model.flat.grad = g
    opt.step()  # the reference's third step, on the reference's gradient
    torch.cuda.synchronize()
    sd = model.state_dict()
    for n in order:
        assert torch.allclose(sd[n].cpu(), torch.from_numpy(rec[f"p3:{n}"]), rtol=1e-5, atol=1e-7), n
    ref_fmt = opt.reference_state_dict()
    for i, n in enumerate(order):
        st = ref_fmt["state"][i]
        assert float(st["step"]) == 3.0
        assert torch.allclose(st["exp_avg"].cpu(), torch.from_numpy(rec[f"st3:{n}:exp_avg"]), rtol=1e-5, atol=1e-9), n
        assert torch.allclose(st["exp_avg_sq"].cpu(), torch.from_numpy(rec[f"st3:{n}:exp_avg_sq"]), rtol=1e-5,
                              atol=1e-12), n


@pytest.mark.gpu
def test_reference_adamw_resumes_fused_state(gpu):
    """The reverse direction: FusedAdamW's reference-format state (after loading the reference's, a round
    trip through the flat buffers) drives a torch.optim.AdamW over the reference's per-tensor parameters to
    the reference's third step."""
    from ergm_amd.optim import FusedAdamW
    rec, order, group, dims = _fixture()
    model = _model(gpu, rec, dims)
    opt = FusedAdamW([model.flat], lr=group["lr"], model=model)
    opt.load_state_dict(_ref_state(rec, order, group))
    saved = opt.reference_state_dict()
    params = [torch.nn.Parameter(torch.from_numpy(rec[f"p2:{n}"]).clone()) for n in order]
    ref_opt = torch.optim.AdamW(params, lr=123.0)
    ref_opt.load_state_dict({"state": {i: {k: (v.cpu() if torch.is_tensor(v) else v) for k, v in s.items()}
                                       for i, s in saved["state"].items()},
                             "param_groups": saved["param_groups"]})
    for p, n in zip(params, order):
        p.grad = torch.from_numpy(rec[f"g3:{n}"])
    ref_opt.step()
    for p, n in zip(params, order):
        assert torch.allclose(p.detach(), torch.from_numpy(rec[f"p3:{n}"]), rtol=1e-6, atol=1e-8), n


@pytest.mark.gpu
def test_trainer_loads_reference_checkpoint(gpu):
    """Trainer.load(resume=True) of a checkpoint whose optim_state_dict is the reference's per-tensor AdamW
    state (src/main.py:107), and Trainer checkpoints write that format."""
    from ergm_amd.optim import FusedAdamW
    from ergm_amd.train import Trainer
    rec, order, group, dims = _fixture()
    model = _model(gpu, rec, dims)
    opt = FusedAdamW([model.flat], lr=group["lr"], model=model)
    ck = {"model_state_dict": {k[3:]: torch.from_numpy(v) for k, v in rec.items() if k.startswith("p2:")},
          "optim_state_dict": _ref_state(rec, order, group), "sched_state_dict": None, "ppl": 12.5, "epoch": 2}
    path = os.path.join(tempfile.mkdtemp(), "ref.ckpt")
    torch.save(ck, path)
    tr = Trainer(model, opt)
    tr.load(path, resume=True)
    assert tr.last_epoch == 2 and tr.best_ppl == 12.5
    st = opt.state[model.flat]
    assert float(st["step"]) == 2.0
    n = "transformer.h.0.mlp.c_fc.weight"
    assert torch.equal(model.view(n, st["exp_avg"]).cpu(), torch.from_numpy(rec[f"st2:{n}:exp_avg"]))
    out = tr.state_dict()["optim_state_dict"]
    assert out["param_groups"][0]["params"] == list(range(len(order)))
    assert torch.equal(out["state"][order.index(n)]["exp_avg"].cpu(), torch.from_numpy(rec[f"st2:{n}:exp_avg"]))
