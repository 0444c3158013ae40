"""Parity margins of the block LayerNorm backward's input precision (the LayerNorms read their
data-gradient GEMM's output rounded to bf16).  Prints the loss error and the max / median gradient rel-L2 of the strict
peaked cross-attention cases (tests/test_gpu_model.py) and the C2 slice for the current ERGM_LN_DY_F32 setting; run it
once with ERGM_LN_DY_F32=0 and once with =1.  Usage: python tools/ln_dy_margin.py"""
import os
import sys

import torch

here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, here)
sys.path.insert(0, os.path.join(here, "tests"))
from oracle import gpt2_oracle as O  # noqa: E402
from test_gpu_model import _grads, _load, _rel, _run, _setup  # noqa: E402

dev = torch.device("cuda:0")
print(f"ERGM_LN_DY_F32={os.environ.get('ERGM_LN_DY_F32', '0')}")
for name in ("xpeak_e128.npz", "xpeak_c2slice.npz", "c2slice_gpt2small_fusion.npz"):
    rec = _load(name)
    ocfg, cfg, P0, model, batch = _setup(rec, dev)
    out = _run(model, batch, dev)
    g = _grads(model)
    if name == "xpeak_e128.npz":
        ref = {k: torch.from_numpy(rec["grad:" + k]) for k in g}
    else:
        _, ref = O.loss_and_grads(P0, ocfg, batch)
    rels = sorted(_rel(g[k], ref[k]) for k in ref)
    lerr = abs(out.loss.item() - float(rec["loss"])) / abs(float(rec["loss"]))
    print(f"{name:32s} loss rel {lerr:.2e}  grad rel-L2 max {rels[-1]:.4e} median {rels[len(rels) // 2]:.4e} "
          f"over {len(rels)} tensors", flush=True)
