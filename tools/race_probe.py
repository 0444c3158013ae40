"""Repeat-run probe for a rare nondeterminism: the fused-optimizer bitwise test at (B, S, E) = (2, 64, 256) once
mismatched in a whole-suite run.  Runs the per-range and the fused optimizer N times each (3 steps, dropout, scheduled
LR, as tests/test_gpu_model.py::test_fused_optimizer_is_bitwise_the_per_range_update) and reports, per run, which
named tensors differ from the first per-range run — so a difference can be pinned on one path and one tensor.
Usage (GPU box): python tools/race_probe.py [N] [B S E]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ergm_amd.config import ERGMConfig  # noqa: E402
from ergm_amd.data import synthetic_batch  # noqa: E402
from ergm_amd.model import GPT2LMHeadModel  # noqa: E402
from ergm_amd.optim import FusedAdamW, get_polynomial_decay_schedule_with_warmup  # noqa: E402
from oracle import gpt2_oracle as O  # noqa: E402


def dirty(dev, value):
    """Fill the caching allocator's free memory with `value` (NaN / a large finite number): a kernel that reads
    an allocation before writing it then shows up as a NaN or a difference."""
    x = torch.full((1 << 28,), value, device=dev)  # 1 GiB, returned to the allocator's cache on del
    torch.cuda.synchronize()
    del x


def one(fuse, B, S, E, dev, fill=None):
    V = 512
    if fill is not None:
        dirty(dev, fill)
    torch.manual_seed(7)
    cfg = ERGMConfig(vocab_size=V, n_embd=E, n_layer=2, n_head=E // 64, n_positions=1024)
    model = GPT2LMHeadModel(cfg, device=dev)
    model.load_state_dict(O.init_params(O.OracleConfig(vocab_size=V, n_embd=E, n_layer=2, n_head=E // 64,
                                                       n_positions=1024), seed=71), strict=False)
    batch = synthetic_batch(B, S, n_turns=3, feat_dim=E, seed=72, vocab_hi=V - 3, sp1=V - 2, sp2=V - 1, eos=V - 4)
    kw = {k: v.to(dev) for k, v in batch.items()}
    opt = FusedAdamW([model.flat], lr=1e-3, model=model, overlap=True, fuse=fuse, keep_grads=True)
    sched = get_polynomial_decay_schedule_with_warmup(opt, 1, 10, power=2.0)
    grads = []
    for _ in range(3):
        opt.zero_grad()
        out = model(input_ids=kw["input_ids"], token_type_ids=kw["token_type_ids"], labels=kw["labels"],
                    emotion_labels=kw["emotion_labels"], caption_ids=kw["caption_ids"], imgs=kw["visual_feat"],
                    auds=kw["audio_feat"])
        out.loss.backward()
        grads.append(model.flat.grad.clone())
        opt.step()
        sched.step()
    torch.cuda.synchronize()
    return model.flat.detach().clone(), grads, model.layout


def diff_names(a, b, layout):
    names = []
    for name, v in layout.views.items():
        n = 1
        for s in v.shape:
            n *= s
        if not torch.equal(a[v.offset:v.offset + n], b[v.offset:v.offset + n]):
            names.append(name)
    return names


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    B, S, E = (int(x) for x in sys.argv[2:5]) if len(sys.argv) > 4 else (2, 64, 256)
    dev = torch.device("cuda:0")
    ref = None
    fills = [None, float("nan"), 1e30, -7.0]
    for it in range(N):
        fill = fills[it % len(fills)]
        for fuse in (False, True):
            p, g, layout = one(fuse, B, S, E, dev, fill)
            if not torch.isfinite(p).all():
                print(f"iter {it} fill {fill} fuse {fuse}: NON-FINITE parameters in "
                      f"{[n for n, v in layout.views.items() if not torch.isfinite(p[v.offset:v.offset + 1]).all()][:8]}",
                      flush=True)
            if ref is None:
                ref = (p, g)
                continue
            bad = diff_names(p, ref[0], layout)
            gbad = [diff_names(x, y, layout) for x, y in zip(g, ref[1])]
            tag = ("fused" if fuse else "per-range") + f" fill={fill}"
            if bad or any(gbad):
                print(f"iter {it} {tag}: params differ in {bad[:8]} ({len(bad)}); grads per step differ in "
                      f"{[x[:4] for x in gbad]}", flush=True)
            else:
                print(f"iter {it} {tag}: identical", flush=True)


if __name__ == "__main__":
    main()
