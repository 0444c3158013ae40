"""How much would HIP-graph capture of the whole training step save?  Times the C2 step eagerly and as a
replayed graph of one captured step (LR frozen at capture time: a timing experiment, not a training
mode).  Usage (GPU box): python tools/graph_experiment.py [step|fwdbwd|fwd]  (what is captured: the whole step,
forward + backward without the optimizer, the training forward alone) [batch] (default 16; 1 = one forward chain)"""
import faulthandler
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    faulthandler.enable()
    from ergm_amd.config import gpt2_small
    from ergm_amd.data import synthetic_batch
    from ergm_amd.model import GPT2LMHeadModel
    from ergm_amd.optim import FusedAdamW
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    model = GPT2LMHeadModel(gpt2_small(), device=dev)
    model.init_weights(seed=0)
    mode = sys.argv[1] if len(sys.argv) > 1 else "step"
    opt = FusedAdamW([model.flat], lr=2e-5, model=model, overlap=mode == "step")  # no updates inside fwdbwd
    bsz = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    b = synthetic_batch(bsz, 128, n_turns=5, seed=1)
    kw = dict(input_ids=b["input_ids"], token_type_ids=b["token_type_ids"], labels=b["labels"],
              emotion_labels=b["emotion_labels"], caption_ids=b["caption_ids"], imgs=b["visual_feat"],
              auds=b["audio_feat"])
    kw = {k: v.to(dev) for k, v in kw.items()}

    def step():
        out = model(**kw)
        if mode == "fwd":
            return out
        opt.zero_grad()
        out.loss.backward()
        if mode == "step":
            opt.step()
        return out

    s = torch.cuda.Stream(dev)
    with torch.cuda.stream(s):
        for _ in range(5):
            step()
    torch.cuda.synchronize()
    K = 30
    t0 = time.perf_counter()
    for _ in range(K):
        step()
    torch.cuda.synchronize()
    eager = (time.perf_counter() - t0) / K * 1e3
    print(f"{mode}: eager {eager:.3f} ms/step; capturing", flush=True)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        step()
    print("captured", flush=True)
    torch.cuda.synchronize()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(K):
        g.replay()
    torch.cuda.synchronize()
    graph = (time.perf_counter() - t0) / K * 1e3
    print(f"eager {eager:.3f} ms/step  graph {graph:.3f} ms/step  ({eager / graph:.3f}x)", flush=True)


if __name__ == "__main__":
    main()
