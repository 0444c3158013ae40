"""Uninitialised-read probe of the executor workspace (GPU box): the trainer test's model and data (tests/
test_gpu_train.py) trained two epochs three times, with every runner allocation made through torch.empty (the
executor workspace, the logits / emotion-logit / loss outputs of each forward) pre-filled with 0x00, 0xFF (NaN for
f32 / bf16) and 0x3F bytes; the three final states must be bitwise equal if no
kernel reads workspace bytes it has not written.  Usage: python tools/ws_probe.py"""
import os
import sys
import types

import torch

here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, here)
sys.path.insert(0, os.path.join(here, "tests"))
import ergm_amd.runtime as R  # noqa: E402
from ergm_amd.train import Trainer  # noqa: E402
from _bitwise import describe  # noqa: E402
from test_gpu_train import _data, _loader, _setup, _state  # noqa: E402

FILL = [None]
proxy = types.SimpleNamespace(**{k: getattr(torch, k) for k in dir(torch) if not k.startswith("__")})


def _empty(*a, **k):
    t = torch.empty(*a, **k)
    if FILL[0] is not None:  # every torch.empty of the runner: the workspace (bytes) and the forward's outputs
        t.view(torch.uint8).fill_(FILL[0]) if t.is_contiguous() and t.numel() else None
    return t


proxy.empty = _empty
R.torch = proxy


def run(fill):
    FILL[0] = fill
    dev = torch.device("cuda:0")
    train_ds, valid_ds = _data(8, 1), _data(3, 2)
    m, o, s = _setup(dev)
    Trainer(m, o, s).train(_loader(train_ds), _loader(valid_ds), 2, log=lambda *_: None)
    torch.cuda.synchronize()
    return _state(m, o), m.layout


base, lay = run(0x00)
for fill in (0xFF, 0x3F):
    st, _ = run(fill)
    for k in base:
        a, b = base[k], st[k]
        same = bool(((a == b) | (torch.isnan(a.float()) & torch.isnan(b.float()))).all()) if a.is_floating_point() \
            else torch.equal(a, b)
        print(f"fill 0x{fill:02X} {k}: {'bitwise equal' if same else describe(b, a, lay)}", flush=True)
