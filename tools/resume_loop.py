"""The trainer resume test (tests/test_gpu_train.py) repeated N times in one process (GPU box): each repetition's
models die with it and are collected at some later point (the model and its overlapped optimizer reference each
other), so later repetitions run beside that teardown.  ``--gc`` collects and synchronises before every repetition.
``--warm S`` first runs S seconds of large GEMMs (the GPU's clocks and temperature after a test suite, no other
state).  ``--scribble`` fills the allocator's cached blocks with random values before every repetition (tensors of
many sizes allocated, filled and freed), so memory a repetition reads without writing holds other values than the
previous repetition left.  Usage: python tools/resume_loop.py N [--gc] [--warm S] [--scribble]"""
import gc
import os
import sys

import torch

here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, here)
sys.path.insert(0, os.path.join(here, "tests"))
from test_gpu_train import test_trainer_epochs_checkpoint_and_resume as resume_test  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 50
collect = "--gc" in sys.argv
dev = torch.device("cuda:0")
if "--warm" in sys.argv:
    import time
    secs = float(sys.argv[sys.argv.index("--warm") + 1])
    A = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)
    t0 = time.time()
    while time.time() - t0 < secs:
        for _ in range(50):
            A.mm(A)
        torch.cuda.synchronize()
    print(f"warmed {secs:.0f} s", flush=True)
scribble = "--scribble" in sys.argv
g = torch.Generator(device=dev).manual_seed(7)
fails = 0
for i in range(n):
    if scribble:
        junk = [torch.randn(int(k), device=dev, generator=g) for k in
                torch.randint(1, 1 << 18, (400,), generator=torch.Generator().manual_seed(i)).tolist()]
        junk += [torch.randn(1 << 22, device=dev, generator=g) for _ in range(8)]
        del junk
    if collect:
        gc.collect()
        torch.cuda.synchronize()
    try:
        resume_test(dev)
    except AssertionError as ex:
        fails += 1
        print(f"repetition {i}: FAILED {str(ex)[:2500]}", flush=True)
print(f"{'gc' if collect else 'scribble' if scribble else 'plain'}: {n - fails}/{n} passed", flush=True)
