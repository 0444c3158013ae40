"""Measure how far the fp8 forward (config 5 scheme) moves the training step from the fp32 oracle,
next to the bf16 path's deviation on the same inputs (used to set the fp8 gates in
tests/test_gpu_c5.py).  Prints one line per (geometry, precision).

    python tools/fp8_parity.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))

from ergm_amd.config import ERGMConfig  # noqa: E402
from ergm_amd.data import synthetic_batch  # noqa: E402
from ergm_amd.model import GPT2LMHeadModel  # noqa: E402
from oracle import gpt2_oracle as O  # noqa: E402


def run(V, E, Lyr, H, Fd, B, S, seed):
    dev = torch.device("cuda:0")
    ocfg = O.OracleConfig(vocab_size=V, n_embd=E, n_layer=Lyr, n_head=H, feat_dim=Fd)
    P0 = O.init_params(ocfg, seed=seed)
    kw = dict(vocab_hi=V - 10, sp1=V - 2, sp2=V - 1, eos=V - 11) if V < 50000 else {}
    batch = synthetic_batch(B, S, n_turns=5, feat_dim=Fd, seed=seed + 1, **kw)
    ref, og = O.loss_and_grads(P0, ocfg, batch)
    for fp8 in (False, True):
        cfg = ERGMConfig(vocab_size=V, n_embd=E, n_layer=Lyr, n_head=H, feat_dim=Fd, fp8=fp8)
        m = GPT2LMHeadModel(cfg, device=dev)
        m.load_state_dict(P0, strict=True)
        b = {k: v.to(dev) for k, v in batch.items()}
        out = m(input_ids=b["input_ids"], token_type_ids=b["token_type_ids"], labels=b["labels"],
                emotion_labels=b["emotion_labels"], caption_ids=b["caption_ids"], imgs=b["visual_feat"],
                auds=b["audio_feat"])
        out.loss.backward()
        torch.cuda.synchronize()
        dl = abs(out.loss.item() - ref["loss"].item()) / abs(ref["loss"].item())
        dlog = (out.logits.float().cpu() - ref["logits"]).abs().max().item()
        rels = []
        for k, r in og.items():
            gk = m.view(k, m.flat.grad).float().cpu()
            rels.append(((gk - r).norm() / r.norm().clamp_min(1e-30)).item())
        rels.sort()
        print(f"E={E} L={Lyr} V={V} B={B} S={S} fp8={fp8}: loss rel {dl:.2e}  logits max|d| {dlog:.4f} "
              f"(|ref| max {ref['logits'].abs().max().item():.3f})  grad rel-L2 median {rels[len(rels) // 2]:.3e} "
              f"p90 {rels[int(0.9 * len(rels))]:.3e} max {rels[-1]:.3e}", flush=True)


if __name__ == "__main__":
    run(500, 128, 2, 2, 64, 3, 64, 31)
    run(50260, 1024, 2, 16, 768, 2, 128, 23)
