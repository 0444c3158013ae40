"""Host enqueue breakdown of the C2 step (GPU box): forward call, backward without / with the overlapped
optimizer hooks, optimizer step and the bench's metric ops, each timed on the host over K steps while
the GPU is held busy by a spin kernel (so no call waits for the device).  Usage: python tools/host_breakdown.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from ergm_amd.config import ERGMConfig  # noqa: E402
from ergm_amd.data import synthetic_batch  # noqa: E402
from ergm_amd.model import GPT2LMHeadModel  # noqa: E402
from ergm_amd.optim import FusedAdamW  # noqa: E402

dev = torch.device("cuda", 0)
cfg = ERGMConfig(n_embd=768, n_layer=12, n_head=12, feat_dim=768)
model = GPT2LMHeadModel(cfg, device=dev)
opt = FusedAdamW([model.flat], lr=2e-5, model=model, overlap=True)
b = synthetic_batch(16, 128, n_turns=5, seed=1000, feat_dim=768)
kw = dict(input_ids=b["input_ids"], token_type_ids=b["token_type_ids"], labels=b["labels"],
          emotion_labels=b["emotion_labels"], caption_ids=b["caption_ids"], imgs=b["visual_feat"], auds=b["audio_feat"])
kw = {k: v.to(dev) for k, v in kw.items()}
acc = torch.zeros(2, device=dev)
cor = torch.zeros(1, device=dev, dtype=torch.int64)
T = {"forward": 0.0, "zero_grad": 0.0, "backward": 0.0, "opt.step": 0.0, "metrics": 0.0}


def step(t):
    t0 = time.perf_counter()
    out = model(**kw)
    t1 = time.perf_counter()
    opt.zero_grad()
    t2 = time.perf_counter()
    out.loss.backward()
    t3 = time.perf_counter()
    opt.step()
    t4 = time.perf_counter()
    acc[0] += out.loss.detach()
    acc[1] += out.loss_lm
    cor.add_((out.emotion_logits.argmax(-1) == kw["emotion_labels"]).sum())
    t5 = time.perf_counter()
    if t:
        for k, a, z in (("forward", t0, t1), ("zero_grad", t1, t2), ("backward", t2, t3), ("opt.step", t3, t4),
                        ("metrics", t4, t5)):
            T[k] += z - a


for _ in range(5):
    step(False)
torch.cuda.synchronize()
K = 10
torch.cuda._sleep(int(2.4e9 * 0.2))
for _ in range(K):
    step(True)
torch.cuda.synchronize()
print({k: round(1000 * v / K, 3) for k, v in T.items()}, "total", round(1000 * sum(T.values()) / K, 3), "ms/step")
# inside the autograd backward: time the runner's backward and the optimizer descriptor
import ergm_amd.runtime as RT  # noqa: E402
from ergm_amd import optim as OP  # noqa: E402
inner = {"runner.backward": 0.0, "native_desc": 0.0}
_rb, _nd = RT.ModelRunner.backward, OP.FusedAdamW._native_desc


def rb(self, *a, **k):
    t0 = time.perf_counter()
    r = _rb(self, *a, **k)
    inner["runner.backward"] += time.perf_counter() - t0
    return r


def nd(self, *a, **k):
    t0 = time.perf_counter()
    r = _nd(self, *a, **k)
    inner["native_desc"] += time.perf_counter() - t0
    return r


RT.ModelRunner.backward, OP.FusedAdamW._native_desc = rb, nd
for k in T:
    T[k] = 0.0
torch.cuda.synchronize()
torch.cuda._sleep(int(2.4e9 * 0.2))
for _ in range(K):
    step(True)
torch.cuda.synchronize()
print({k: round(1000 * v / K, 3) for k, v in T.items()}, {k: round(1000 * v / K, 3) for k, v in inner.items()})
# native calls alone: the runner's backward without the optimizer hooks
runner = next(iter(model._runners.values()))
gl = torch.ones(1, device=dev)
torch.cuda._sleep(int(2.4e9 * 0.2))
tb = 0.0
for _ in range(K):
    model(**kw)
    t0 = time.perf_counter()
    runner.backward(gl, None)
    tb += time.perf_counter() - t0
torch.cuda.synchronize()
print("runner.backward without optimizer hooks", round(1000 * tb / K, 3), "ms")
