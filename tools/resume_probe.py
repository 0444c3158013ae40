"""Resume divergence probe (GPU box): the trainer test's flow (tests/test_gpu_train.py) with the third epoch of the
uninterrupted model m1 and of the resumed model m3 run in lockstep, batch by batch, comparing loss and master after
every step; repeated up to R times, stopping at the first divergence.  Usage: python tools/resume_probe.py [R]"""
import os
import sys
import tempfile

import torch

here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, here)
sys.path.insert(0, os.path.join(here, "tests"))
from ergm_amd.dataset import DevicePrefetcher  # noqa: E402
from ergm_amd.train import Trainer  # noqa: E402
from _bitwise import describe  # noqa: E402
from test_gpu_train import _data, _loader, _setup, _state  # noqa: E402

dev = torch.device("cuda:0")
R = int(sys.argv[1]) if len(sys.argv) > 1 else 4
train_ds, valid_ds = _data(8, 1), _data(3, 2)


def step(model, opt, sched, batch):
    kw = dict(input_ids=batch["input_ids"], token_type_ids=batch["token_type_ids"], labels=batch["labels"],
              emotion_labels=batch["emotion_labels"], caption_ids=batch["caption_ids"],
              imgs=batch.get("visual_feat"), auds=batch.get("audio_feat"))
    out = model(**kw)
    opt.zero_grad()
    out.loss.backward()
    opt.step()
    sched.step()
    return out.loss.detach().clone()


for rep in range(R):
    tmp = tempfile.mkdtemp()
    m1, o1, s1 = _setup(dev)
    t1 = Trainer(m1, o1, s1, ckpt_dir=tmp)
    t1.validation(_loader(valid_ds))
    t1.train(_loader(train_ds), _loader(valid_ds), 2, log=lambda *_: None)
    path = os.path.join(tmp, "mid.ckpt")
    t1.save(path)
    m3, o3, s3 = _setup(dev)
    t3 = Trainer(m3, o3, s3)
    t3.load(path)
    m3.refresh_bf16()
    torch.cuda.synchronize()
    a, b = _state(m1, o1), _state(m3, o3)
    bad = [k for k in a if not torch.equal(a[k], b[k])]
    g1, g3 = o1.param_groups[0], o3.param_groups[0]
    print(f"rep {rep}: after load: differ {bad}; lr {g1['lr']!r} vs {g3['lr']!r}; step "
          f"{float(o1.state[m1.flat]['step'])} vs {float(o3.state[m3.flat]['step'])}; sched "
          f"{s1.last_epoch} vs {s3.last_epoch}", flush=True)
    m1.train(); m3.train()
    diverged = False
    for i, batch in enumerate(DevicePrefetcher(_loader(train_ds), dev)):
        l1 = step(m1, o1, s1, batch)
        l3 = step(m3, o3, s3, batch)
        torch.cuda.synchronize()
        same_loss = torch.equal(l1, l3)
        if not same_loss or not torch.equal(m1.flat, m3.flat):
            print(f"rep {rep}: epoch-3 step {i} (S={batch['input_ids'].shape[1]}): loss {l1.item():.9g} vs "
                  f"{l3.item():.9g}; master {describe(m3.flat.detach(), m1.flat.detach(), m1.layout)}", flush=True)
            diverged = True
            break
    print(f"rep {rep}: {'DIVERGED' if diverged else 'lockstep bitwise equal'}", flush=True)
    if diverged:
        break
