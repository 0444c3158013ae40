"""Isolated attention timings at the training configs' shapes (HIP-graph replay, no concurrency), with
algorithmic TFLOP/s: forward 4·B·H·Sq·Sk·64 FLOP (half of it for causal), backward 2.5x the forward
(dV, dP, dS·K for dQ, dSᵀ·Q for dK; the recomputed QKᵀ not counted).  Usage (GPU box):
python tools/attn_bench.py [--generic] [--ns 2,3,4] [--only c4]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ergm_amd import _lib as L  # noqa: E402
from ergm_amd import ops  # noqa: E402

REPS = 20
SHAPES = {"c2": (16, 128, 12), "c4": (8, 512, 12), "c5": (32, 128, 16)}


def timed(fn):
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(REPS):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / (5 * REPS) * 1e3


def main():
    lib = L.load()
    arg = lambda k, d: sys.argv[sys.argv.index(k) + 1] if k in sys.argv else d  # noqa: E731
    for ns in [int(x) for x in arg("--ns", "0").split(",")]:
        L.check(lib.ergm_attn_tune(int("--generic" in sys.argv) | (ns << 4)), "attn_tune")
        if ns:
            print(f"ring stages {ns}")
        run(arg("--only", None))


def run(only):
    dev = torch.device("cuda:0")
    for name, (B, S, H) in SHAPES.items():
        if only and name != only:
            continue
        E = 64 * H
        T = B * S
        for causal in (True, False):
            torch.manual_seed(0)
            qkv = torch.randn(T, 3 * E, device=dev).bfloat16()
            q, k, v = qkv[:, :E], qkv[:, E:2 * E], qkv[:, 2 * E:]
            o, lse = ops.attn_fwd(q, k, v, B, H, S, S, causal)
            do = torch.randn(T, E, device=dev).bfloat16()
            fl = 4.0 * B * H * S * S * 64 * (0.5 if causal else 1.0)
            tf = timed(lambda: ops.attn_fwd(q, k, v, B, H, S, S, causal))
            tb = timed(lambda: ops.attn_bwd(q, k, v, o, do, lse, B, H, S, S, causal))
            tag = "causal" if causal else "cross "
            print(f"{name} B={B:2d} S={S} H={H} {tag}: fwd {tf:7.2f} us {fl / tf / 1e6:6.1f} TF/s   "
                  f"bwd {tb:7.2f} us {2.5 * fl / tb / 1e6:6.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
