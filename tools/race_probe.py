"""Timing-perturbed resume probe (GPU box): the trainer test's flow (tests/test_gpu_train.py) — two epochs, a
checkpoint, the third epoch — with the resumed third epoch repeated under perturbations that move the relative
timing of the caller's stream, the executor's own streams and the host, each run compared bitwise with the
unperturbed third epoch.  A race between the executor's streams and memory the caller's allocator recycles
shows up as a mismatch under some perturbation.  Usage: python tools/race_probe.py [reps_per_mode]

Modes (applied between the trainer's steps, seeded per repetition):
  none   no perturbation
  sleep  host sleeps 0-3 ms (the GPU drains, the host falls behind)
  busy   0-3 large GEMMs on the caller's stream (the caller's stream runs late against the executor's)
  churn  0-64 small and large tensors allocated, written and freed on the caller's stream (recycled blocks)
  side   GEMMs on a second torch stream, concurrent with the step (CUs shared unevenly)"""
import os
import random
import sys
import tempfile
import time

import torch

here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, here)
sys.path.insert(0, os.path.join(here, "tests"))
from ergm_amd.train import Trainer  # noqa: E402
from _bitwise import describe  # noqa: E402
from test_gpu_train import _data, _loader, _setup  # noqa: E402

dev = torch.device("cuda:0")


def perturbed(loader, mode, rng, A, other):
    for batch in loader:
        if mode == "sleep":
            time.sleep(rng.random() * 3e-3)
        elif mode == "busy":
            for _ in range(rng.randrange(4)):
                A.mm(A)
        elif mode == "churn":
            keep = []
            for _ in range(rng.randrange(65)):
                n = rng.choice((1, 3, 7, 128, 4096, 1 << 18))
                keep.append(torch.empty(n, device=dev).fill_(rng.random()))
            del keep
        elif mode == "side":
            with torch.cuda.stream(other):
                for _ in range(rng.randrange(4)):
                    A.mm(A)
        yield batch



def main(R=8, modes=("none", "sleep", "busy", "churn", "side")):
    train_ds, valid_ds = _data(8, 1), _data(3, 2)
    A = torch.randn(2048, 2048, device=dev)
    other = torch.cuda.Stream(dev)
    tmp = tempfile.mkdtemp()
    m1, o1, s1 = _setup(dev)
    t1 = Trainer(m1, o1, s1, ckpt_dir=tmp)
    t1.validation(_loader(valid_ds))
    t1.train(_loader(train_ds), _loader(valid_ds), 2, log=lambda *_: None)
    path = os.path.join(tmp, "mid.ckpt")
    t1.save(path)
    first = t1.train_epoch(_loader(train_ds))
    torch.cuda.synchronize()
    ref = m1.flat.detach().clone()
    print(f"reference third epoch: loss {first.loss:.9g}", flush=True)
    bad = 0
    for mode in modes:
        n_bad = 0
        for rep in range(R):
            rng = random.Random(1000 * rep + len(mode))
            m3, o3, s3 = _setup(dev)
            t3 = Trainer(m3, o3, s3)
            t3.load(path)
            again = t3.train_epoch(perturbed(_loader(train_ds), mode, rng, A, other))
            torch.cuda.synchronize()
            if not torch.equal(m3.flat, ref) or again.loss != first.loss:
                n_bad += 1
                print(f"{mode} rep {rep}: DIVERGED loss {again.loss:.9g}; master {describe(m3.flat.detach(), ref, m1.layout)}",
                      flush=True)
            del m3, o3, s3, t3
        print(f"mode {mode}: {R - n_bad}/{R} bitwise equal", flush=True)
        bad += n_bad
    print("RESULT", "all equal" if bad == 0 else f"{bad} diverged", flush=True)
    return bad


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 8)
