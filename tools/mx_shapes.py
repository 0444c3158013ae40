"""Isolated timing of the config-5 forward GEMM shapes (per forward chain, M = 2048): MX-fp8 per tile
configuration, per-row fp8, and bf16 (default plan).  python tools/mx_shapes.py [M]"""
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))

from ergm_amd import _lib as L
from ergm_amd import ops

M = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
dev = torch.device("cuda:0")
lib = L.load()
SHAPES = [("qkv", 3072, 1024, L.EPI_BIAS), ("proj", 1024, 1024, L.EPI_BIAS_RESID), ("fc", 4096, 1024, L.EPI_BIAS_GELU),
          ("mproj", 1024, 4096, L.EPI_BIAS_RESID), ("crossq", 1024, 1024, L.EPI_BIAS)]


def timeit(fn, reps=50):
    for _ in range(5):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / reps


for name, N, K, epi in SHAPES:
    g = torch.Generator(device=dev).manual_seed(0)
    A = (torch.randn(M, K, device=dev, generator=g)).bfloat16()
    W = (torch.randn(K, N, device=dev, generator=g) * 0.02).bfloat16()
    bias = torch.zeros(N, device=dev)
    ob = epi != L.EPI_BIAS_RESID
    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16 if ob else torch.float32)
    aux = torch.zeros(M, N, device=dev) if epi == L.EPI_BIAS_RESID else None
    aux_out = torch.empty(M, N, device=dev, dtype=torch.bfloat16) if epi == L.EPI_BIAS_GELU else None
    qa, sa = ops.quant_rows_mx(A)
    wt, sw = ops.quant_weight_mx(W)
    qr, sr = ops.quant_rows_fp8(A)
    wr, swr = ops.quant_weight_fp8(W)
    fl = 2.0 * M * N * K
    res = {}
    for cfg in range(-1, 5):
        L.check(lib.ergm_gemm_f8_tune(cfg), "tune")
        t = timeit(lambda: ops.gemm_mx(qa, sa, wt, sw, out=out, epilogue=epi, bias=bias, aux=aux, aux_out=aux_out))
        t8 = timeit(lambda: ops.gemm_f8(qr, sr, wr, swr, out=out, epilogue=epi, bias=bias, aux=aux, aux_out=aux_out))
        res[cfg] = (t, t8)
    lib.ergm_gemm_f8_tune(-1)
    tb = timeit(lambda: ops.gemm(A, W, M, N, K, L.MK, L.KN, out=out, epilogue=epi, bias=bias, aux=aux,
                                 aux_out=aux_out))
    line = " ".join(f"c{c}:{t:6.1f}/{t8:6.1f}" for c, (t, t8) in res.items())
    print(f"{name:6s} M={M} N={N} K={K}: bf16 {tb:6.1f} us ({fl / tb / 1e6:5.0f} TF/s) | mx/row {line} "
          f"| best mx {fl / min(v[0] for v in res.values()) / 1e6:5.0f} TF/s", flush=True)
