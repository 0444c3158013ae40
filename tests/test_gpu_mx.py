"""MX-fp8 (OCP microscaling) path of config 5 on the GPU, through the C-ABI: e4m3fn elements with an e8m0
scale per 32-element K block, consumed by v_mfma_scale_f32_16x16x128_f8f6f4 itself.

* quantisers (rows; weights into their transpose and, for the fp8 data-gradient GEMMs, their row form): bit-exact
  against a torch restatement of the rule
  (block exponent e = the smallest integer with max|block| <= 448·2^e, from the bits of the maximum; values
  scaled by 2^-e exactly, then torch's float8_e4m3fn cast: round to nearest even);
* ergm_gemm_mx: exact MX inputs with random block scales, f32 accumulation -> against an fp64 product of the
  dequantised operands (rel 5e-5), every tile configuration, ragged M / N;
* the GELU / GELU' epilogues' MX copy of their bf16 output is bit-identical to quantising that output afterwards.
Scales travel in the library's K-step-major layout (ops.mx_tile / mx_untile convert).
The model-level fp8 gates (tests/test_gpu_c5.py) run on this path by default (ERGM_FP8_MX=1).
"""
import pytest
import torch

from ergm_amd import _lib as L
from ergm_amd import ops

pytestmark = pytest.mark.gpu
E4M3 = torch.float8_e4m3fn


def mx_ref(X: torch.Tensor):
    """(Q [R, C] uint8, S [R, C/32] uint8) of rows X [R, C] (C % 32 == 0)."""
    X = X.float()
    R, Cc = X.shape
    Xb = X.reshape(R, Cc // 32, 32)
    am = Xb.abs().amax(-1).contiguous()
    bits = am.view(torch.int32)
    ea = ((bits >> 23) & 0xFF) - 127
    e = ea - 8 + ((bits & 0x7FFFFF) > 0x600000).to(torch.int32)
    eb = torch.where(am == 0, torch.full_like(e, 127), (e + 127).clamp(0, 254))
    inv = torch.pow(2.0, (127 - eb).double()).float()
    q = (Xb * inv[..., None]).clamp(-448, 448).to(E4M3)
    return q.view(torch.uint8).reshape(R, Cc), eb.to(torch.uint8)


def mx_dequant(Q: torch.Tensor, S: torch.Tensor) -> torch.Tensor:
    R, Cc = Q.shape
    v = Q.view(E4M3).double().reshape(R, Cc // 32, 32)
    return (v * torch.pow(2.0, S.double() - 127)[..., None]).reshape(R, Cc)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("rows,cols,ld", [(64, 1024, 1032), (37, 4096, 4104), (5, 96, 104)])
def test_quant_rows_mx_bit_exact(gpu, dtype, rows, cols, ld):
    g = torch.Generator().manual_seed(rows + cols)
    X = torch.randn(rows, ld, generator=g) * torch.logspace(-3, 2, rows)[:, None]
    X[0] = 0.0                      # zero blocks -> scale 1
    X[1, :32] = 448.0 * 2.0 ** -3   # a block whose maximum is exactly 448·2^e
    X[1, 32:64] = 1.8               # mantissa above 1.75: the next exponent up
    X = X.to(dtype)
    q, s = ops.quant_rows_mx(X.to(gpu), cols)
    rq, rs = mx_ref(X[:, :cols])
    s = ops.mx_untile(s.cpu(), rows, cols // 32)
    assert torch.equal(s, rs)
    assert torch.equal(q.cpu(), rq)
    # no element saturates and the dequantised values are within e4m3's half-ulp (2^-4 relative)
    deq = mx_dequant(q.cpu(), s)
    ref = X[:, :cols].double()
    assert ((deq - ref).abs() <= ref.abs() * 2.0 ** -4 + 2.0 ** -9 * ref.abs().amax()).all()


@pytest.mark.parametrize("K,N", [(1024, 3072), (4096, 1024), (128, 192)])
def test_quant_weight_mx_bit_exact(gpu, K, N):
    g = torch.Generator().manual_seed(K + N)
    W = torch.randn(K, N, generator=g) * 0.02
    W[:, 5] = 0.0
    W[:32, 7] *= 1000.0
    W[9, 64:96] = 0.0
    W = W.bfloat16()
    Wt, s, Wr, sr = ops.quant_weight_mx(W.to(gpu), row_form=True)
    rq, rs = mx_ref(W.t().contiguous())
    assert torch.equal(ops.mx_untile(s.cpu(), N, K // 32), rs)
    assert torch.equal(Wt.cpu(), rq)
    rq, rs = mx_ref(W)  # the row form: W's rows along N
    assert torch.equal(ops.mx_untile(sr.cpu(), K, N // 32), rs)
    assert torch.equal(Wr.cpu(), rq)


def _mx_operand(rows, K, g):
    q = (torch.randn(rows, K, generator=g) * 3.0).clamp(-448, 448).to(E4M3).view(torch.uint8)
    s = torch.randint(120, 135, (rows, K // 32), generator=g, dtype=torch.int32).to(torch.uint8)
    return q, s


N_F8_CFGS = 5  # kF8Cfgs in gemm.hip (shared by the MX kernel)


@pytest.mark.parametrize("cfg", [-1] + list(range(N_F8_CFGS)))
@pytest.mark.parametrize("M,N,K", [(256, 384, 512), (200, 136, 256), (2048, 1024, 1024), (64, 4096, 128)])
def test_gemm_mx_matches_fp64(gpu, cfg, M, N, K):
    lib = L.load()
    g = torch.Generator().manual_seed(M + N + K + cfg)
    A8, sa = _mx_operand(M, K, g)
    B8, sb = _mx_operand(N, K, g)
    ref = mx_dequant(A8, sa) @ mx_dequant(B8, sb).t()
    try:
        L.check(lib.ergm_gemm_f8_tune(cfg), "tune")
        out = ops.gemm_mx(A8.to(gpu), ops.mx_tile(sa).to(gpu), B8.to(gpu), ops.mx_tile(sb, N + 8).to(gpu))
        torch.cuda.synchronize()
    finally:
        lib.ergm_gemm_f8_tune(-1)
    err = ((out.double().cpu() - ref).norm() / ref.norm()).item()
    assert err < 5e-5, err


def test_gemm_mx_epilogues_and_gelu_mx_copy(gpu):
    M, N, K = 512, 1024, 768
    g = torch.Generator().manual_seed(3)
    A8, sa = _mx_operand(M, K, g)
    B8, sb = _mx_operand(N, K, g)
    sa = (sa.int() - 8).to(torch.uint8)  # keep the products O(1) for the GELU
    sb = (sb.int() - 8).to(torch.uint8)
    bias = torch.randn(N, generator=g)
    res = torch.randn(M, N, generator=g)
    v = mx_dequant(A8, sa) @ mx_dequant(B8, sb).t() + bias.double()
    dev = lambda t: t.to(gpu)  # noqa: E731
    a8, b8, xa, xb = dev(A8), dev(B8), dev(ops.mx_tile(sa)), dev(ops.mx_tile(sb))
    out = ops.gemm_mx(a8, xa, b8, xb, epilogue=L.EPI_BIAS_RESID, bias=dev(bias), aux=dev(res))
    assert ((out.double().cpu() - (v + res.double())).norm() / (v + res.double()).norm()).item() < 5e-5
    pre = torch.empty(M, N, dtype=torch.bfloat16, device=gpu)
    act = torch.empty(M, N + 8, dtype=torch.bfloat16, device=gpu)[:, :N]
    q = torch.empty(M, N, dtype=torch.uint8, device=gpu)
    qs = torch.empty(N // 128, M + 16, 4, dtype=torch.uint8, device=gpu)
    ops.gemm_mx(a8, xa, b8, xb, out=act, epilogue=L.EPI_BIAS_GELU, bias=dev(bias), aux_out=pre, q_out=q, q_sc=qs)
    vv = v.clone().requires_grad_(True)
    gelu = 0.5 * vv * (1 + torch.tanh((2 / torch.pi) ** 0.5 * (vv + 0.044715 * vv ** 3)))
    gelu.sum().backward()
    gelu = gelu.detach()
    assert (pre.double().cpu() - vv.grad).abs().max().item() <= 8e-3 * vv.grad.abs().max().item()
    assert (act.double().cpu() - gelu).abs().max().item() <= 8e-3 * gelu.abs().max().item()
    # the epilogue's MX copy is exactly the MX quantisation of the bf16 output it stored
    rq, rs = mx_ref(act.cpu())
    assert torch.equal(ops.mx_untile(qs.cpu(), M, N // 32), rs)
    assert torch.equal(q.cpu(), rq)
    outb = ops.gemm_mx(a8, xa, b8, xb, out_dtype=torch.bfloat16, epilogue=L.EPI_BIAS, bias=dev(bias))
    assert ((outb.double().cpu() - v).norm() / v.norm()).item() < 4e-3
    # GELU' (the fp8 data-gradient path's mlp c_proj dX): C = (A·Bᵀ) · aux, with the MX copy of C for the c_fc dX
    dg = (torch.rand(M, N, generator=g) * 1.2 - 0.1).bfloat16()
    gb = torch.empty(M, N, dtype=torch.bfloat16, device=gpu)
    ops.gemm_mx(a8, xa, b8, xb, out=gb, epilogue=L.EPI_GELU_BWD, aux=dev(dg), q_out=q, q_sc=qs)
    vb = (v - bias.double()) * dg.double()
    assert ((gb.double().cpu() - vb).norm() / vb.norm()).item() < 4e-3
    rq, rs = mx_ref(gb.cpu())
    assert torch.equal(ops.mx_untile(qs.cpu(), M, N // 32), rs)
    assert torch.equal(q.cpu(), rq)


def test_gemm_mx_rejects_bad_arguments(gpu):
    a = torch.zeros(64, 128, dtype=torch.uint8, device=gpu)
    s = torch.zeros(1, 64, 4, dtype=torch.uint8, device=gpu)
    with pytest.raises(ValueError):
        ops.gemm_mx(a[:, :100], s, a[:, :100], s)  # K = 100 is not a multiple of 128
    q = torch.zeros(64, 64, dtype=torch.uint8, device=gpu)
    with pytest.raises(ValueError):  # an MX copy of the output needs the GELU epilogue
        ops.gemm_mx(a, s, a, s, out_dtype=torch.bfloat16, epilogue=L.EPI_BIAS,
                    bias=torch.zeros(64, device=gpu), q_out=q, q_sc=s)
