"""VALU passes are bitwise the same whether or not MFMA waves share their CUs (round 6).

The round-5 trainer-test divergence was the AdamW pass computing a wrong low half of a packed-FP32 pair (float4
components 0 / 2) in lanes 48-63 when a GEMM's MFMA waves ran on the same CUs: on gfx950 with ROCm 7.2 a
v_pk_{mul,add}_f32 beside another wave's MFMAs can return wrong results (tools/adamw_hazard.hip: ~1e-3 of the pass's
words beside MFMA waves, 0 alone).  The library is built without packed FP32 instructions (ergm_amd/build.py).  These
tests run the element passes of the training step alone and then repeatedly with large GEMMs in flight on a second
stream, and require every repetition to be bitwise the lone result (the unfixed AdamW failed this in every repetition).
"""
import pytest
import torch

from ergm_amd import _lib as L
from ergm_amd import ops
from _bitwise import assert_bitwise

pytestmark = pytest.mark.gpu
REPS = 12


def _pressure(dev):
    """Two 4096^3 bf16 GEMMs on their own stream (about 0.2 ms of MFMA waves on every CU)."""
    a = torch.randn(4096, 4096, device=dev).bfloat16()
    b = torch.randn(4096, 4096, device=dev).bfloat16()
    c = torch.empty(4096, 4096, device=dev)
    st = torch.cuda.Stream(dev)

    def launch():
        st.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(st):
            for _ in range(2):
                ops.gemm(a, b, 4096, 4096, 4096, L.MK, L.NK, out=c)
    return launch, st


def test_adamw_bitwise_beside_mfma_waves(gpu):
    n = 4 << 20
    g = torch.Generator(device=gpu).manual_seed(3)
    p0 = torch.randn(n, device=gpu, generator=g) * 0.04
    gr = torch.randn(n, device=gpu, generator=g) * 2e-3
    m0 = torch.randn(n, device=gpu, generator=g) * 1e-3
    v0 = torch.rand(n, device=gpu, generator=g) * 1e-6

    def run(pressure=None):
        p, m, v = p0.clone(), m0.clone(), v0.clone()
        sh = torch.empty(n, dtype=torch.bfloat16, device=gpu)
        if pressure is not None:
            pressure()
        for a in range(0, n, 232704):  # the trainer test's bucket size: 114 workgroups per launch
            b = min(a + 232704, n)
            ops.adamw_step(p[a:b], gr[a:b], m[a:b], v[a:b], sh[a:b], 5.8e-4, 0.9, 0.999, 1e-8, 0.01, 12)
        return p, m, v, sh

    ref = run()
    launch, st = _pressure(gpu)
    for r in range(REPS):
        got = run(launch)
        for name, x, y in zip(("param", "exp_avg", "exp_avg_sq", "shadow"), got, ref):
            assert_bitwise(x, y, f"AdamW beside MFMA waves, repetition {r}: {name}")
    torch.cuda.current_stream(gpu).wait_stream(st)


def test_layernorm_bitwise_beside_mfma_waves(gpu):
    rows, E = 8192, 768
    g = torch.Generator(device=gpu).manual_seed(4)
    x = torch.randn(rows, E, device=gpu, generator=g)
    gamma = 1 + 0.1 * torch.randn(E, device=gpu, generator=g)
    beta = 0.1 * torch.randn(E, device=gpu, generator=g)
    dy = torch.randn(rows, E, device=gpu, generator=g)

    def run(pressure=None):
        if pressure is not None:
            pressure()
        y, mean, rstd = ops.layernorm_fwd(x, gamma, beta)
        dres = torch.zeros(rows, E, device=gpu)
        dres, db, dg, dbe = ops.layernorm_bwd(dy, x, mean, rstd, gamma, dres)
        return y, mean, rstd, dres, db, dg, dbe

    ref = run()
    launch, st = _pressure(gpu)
    names = ("y", "mean", "rstd", "dres", "dres_bf16", "dgamma", "dbeta")
    for r in range(REPS):
        for name, a, b in zip(names, run(launch), ref):
            assert_bitwise(a, b, f"LayerNorm beside MFMA waves, repetition {r}: {name}")
    torch.cuda.current_stream(gpu).wait_stream(st)
