"""Host-side profile of the C2 training step enqueue (cProfile over K steps after warm-up): where the
Python/ctypes time of bench.py's step goes.  Usage (GPU box): python tools/host_profile.py [steps]"""
import cProfile
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from ergm_amd.config import ERGMConfig  # noqa: E402
from ergm_amd.data import synthetic_batch  # noqa: E402
from ergm_amd.model import GPT2LMHeadModel  # noqa: E402
from ergm_amd.optim import FusedAdamW, get_polynomial_decay_schedule_with_warmup  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
dev = torch.device("cuda", 0)
cfg = ERGMConfig(n_embd=768, n_layer=12, n_head=12, feat_dim=768)
model = GPT2LMHeadModel(cfg, device=dev)
model.init_weights(seed=0)
opt = FusedAdamW([model.flat], lr=2e-5, model=model, overlap=True)
sched = get_polynomial_decay_schedule_with_warmup(opt, num_warmup_steps=2, num_training_steps=K + 10, power=2)
b = synthetic_batch(16, 128, n_turns=5, seed=1000, feat_dim=768)
kw = dict(input_ids=b["input_ids"], token_type_ids=b["token_type_ids"], labels=b["labels"],
          emotion_labels=b["emotion_labels"], caption_ids=b["caption_ids"], imgs=b["visual_feat"], auds=b["audio_feat"])
kw = {k: v.to(dev) for k, v in kw.items()}
loss_acc = torch.zeros(2, device=dev)
correct = torch.zeros(1, device=dev, dtype=torch.int64)


def step():
    out = model(**kw)
    opt.zero_grad()
    out.loss.backward()
    opt.step()
    sched.step()
    loss_acc[0] += out.loss.detach()
    loss_acc[1] += out.loss_lm
    correct.add_((out.emotion_logits.argmax(-1) == kw["emotion_labels"]).sum())


for _ in range(5):
    step()
torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
for _ in range(K):
    step()
pr.disable()
torch.cuda.synchronize()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(30)
st.sort_stats("cumtime").print_stats(40)
