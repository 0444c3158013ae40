"""Per-kernel parity on the GPU: every HIP kernel against a plain PyTorch fp32/fp64 reference of the
same op on the same (seeded) inputs, called through the C-ABI (ergm_amd.ops → libergm_hip.so)."""
import math

import pytest
import torch
import torch.nn.functional as F

from ergm_amd import _lib as L
from ergm_amd import ops

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def _bf(x):
    return x.to(torch.bfloat16)


def _mat(A, layout_rowK, M, K):
    """logical [M,K] from storage"""
    return A.float() if layout_rowK else A.float().t()


GEMM_SHAPES = [(256, 256, 128), (2048, 2304, 768), (2048, 768, 3072), (96, 200, 72), (64, 50304, 128),
               (768, 768, 2048), (200, 96, 1024), (8, 24, 16)]


@pytest.mark.parametrize("M,N,K", GEMM_SHAPES)
@pytest.mark.parametrize("al,bl", [(L.MK, L.NK), (L.MK, L.KN), (L.KM, L.NK), (L.KM, L.KN)])
def test_gemm_layouts(gpu, M, N, K, al, bl):
    g = torch.Generator(device="cpu").manual_seed(M * 7 + N * 3 + K + al * 2 + bl)
    Am = torch.randn(M, K, generator=g)
    Bm = torch.randn(K, N, generator=g)
    A = _bf(Am if al == L.MK else Am.t().contiguous()).to(gpu)
    B = _bf(Bm.t().contiguous() if bl == L.NK else Bm).to(gpu)
    ref = _bf(Am).double() @ _bf(Bm).double()
    out = ops.gemm(A, B, M, N, K, al, bl, out_dtype=torch.float32)
    assert _rel(out.cpu(), ref) < 1e-5
    outb = ops.gemm(A, B, M, N, K, al, bl, out_dtype=torch.bfloat16)
    assert _rel(outb.float().cpu(), ref) < 6e-3


N_CFGS = 47  # kCfgs in gemm.hip (ergm_gemm_tune rejects an index past the table); 38-46: 32x32x16 MFMA


@pytest.mark.parametrize("cfg", range(N_CFGS))
def test_gemm_every_pipelined_config(gpu, cfg):
    """Each pipelined / warp-specialised tile configuration, forced through ergm_gemm_tune, on ragged
    M/N edges, all four operand layouts, with and without split-K."""
    lib = L.load()
    M, N, K = 328, 392, 512
    g = torch.Generator(device="cpu").manual_seed(cfg)
    Am, Bm = torch.randn(M, K, generator=g), torch.randn(K, N, generator=g)
    ref = _bf(Am).double() @ _bf(Bm).double()
    try:
        for split in (1, 2):
            L.check(lib.ergm_gemm_tune(cfg, split), "tune")
            for al, bl in ((L.MK, L.NK), (L.MK, L.KN), (L.KM, L.NK), (L.KM, L.KN)):
                A = _bf(Am if al == L.MK else Am.t().contiguous()).to(gpu)
                B = _bf(Bm.t().contiguous() if bl == L.NK else Bm).to(gpu)
                out = ops.gemm(A, B, M, N, K, al, bl, out_dtype=torch.float32, split_k=split)
                assert _rel(out.cpu(), ref) < 1e-5, (split, al, bl)
        L.check(lib.ergm_gemm_tune(cfg, 1), "tune")
        W = _bf(Bm).to(gpu)
        bias = torch.randn(N, device=gpu)
        out = ops.gemm(_bf(Am).to(gpu), W, M, N, K, L.MK, L.KN, epilogue=L.EPI_BIAS, bias=bias)
        assert _rel(out.cpu(), ref + bias.double().cpu()) < 1e-5
    finally:
        L.check(lib.ergm_gemm_tune(-1, 0), "tune")
    with pytest.raises(ValueError):
        L.check(lib.ergm_gemm_tune(N_CFGS, 1), "tune")


@pytest.mark.parametrize("split", [2, 3, 5])
def test_gemm_split_k(gpu, split):
    M, N, K = 192, 320, 2048
    A = torch.randn(M, K, device=gpu).bfloat16()
    B = torch.randn(N, K, device=gpu).bfloat16()
    ref = A.double() @ B.double().t()
    out = ops.gemm(A, B, M, N, K, L.MK, L.NK, split_k=split)
    assert _rel(out, ref) < 1e-5
    # split-K is deterministic: same result twice, bit for bit
    out2 = ops.gemm(A, B, M, N, K, L.MK, L.NK, split_k=split)
    assert torch.equal(out, out2)


@pytest.mark.parametrize("M,N,K,split,cfg", [(768, 2304, 2048, 1, -1), (768, 768, 4096, 0, -1),
                                               (200, 136, 1000, 1, -1), (256, 512, 2048, 3, -1),
                                               (256, 512, 1024, 1, 0), (256, 512, 1024, 2, 2),
                                               (256, 512, 1024, 1, 16)])
def test_gemm_bias_grad(gpu, M, N, K, split, cfg):
    """Weight gradient + its Conv1D bias gradient in one GEMM (ergm_gemm_desc.bias_grad): dW = Xᵀ·dY and
    db = Σ_t dY[t] (the in-kernel column sums of the pipelined kernels, their split-K partials, and the
    column-sum pass of the kernels without it: register-staged for K % 64 != 0, warp-specialised cfg 16),
    against fp64; bitwise reproducible."""
    g = torch.Generator(device="cpu").manual_seed(M + N + K)
    X = (torch.randn(K, M, generator=g) * 0.5).to(gpu, torch.bfloat16)   # [tokens][in]  (KM)
    dY = (torch.randn(K, N, generator=g) * 0.5).to(gpu, torch.bfloat16)  # [tokens][out] (KN)
    L.check(L.load().ergm_gemm_tune(cfg, split if cfg >= 0 else 0), "tune")
    try:
        db = torch.full((N,), float("nan"), device=gpu)
        dW = ops.gemm(X, dY, M, N, K, a_layout=L.KM, b_layout=L.KN, split_k=split if cfg < 0 else 0, bias_grad=db)
        db2 = torch.full((N,), float("nan"), device=gpu)
        ops.gemm(X, dY, M, N, K, a_layout=L.KM, b_layout=L.KN, split_k=split if cfg < 0 else 0, bias_grad=db2)
    finally:
        L.load().ergm_gemm_tune(-1, 0)
    torch.cuda.synchronize()
    ref_w = X.double().t() @ dY.double()
    ref_b = dY.double().sum(0)
    assert ((dW.double() - ref_w).norm() / ref_w.norm()).item() < 1e-5
    assert ((db.double() - ref_b).abs() / (ref_b.abs() + 1.0)).max().item() < 1e-4
    assert torch.equal(db, db2)
    with pytest.raises(ValueError):  # other layouts / epilogues reject it
        ops.gemm(X.t().contiguous(), dY, M, N, K, a_layout=L.MK, b_layout=L.KN, bias_grad=db)


def test_gemm_epilogues(gpu):
    M, N, K = 256, 384, 192
    A = torch.randn(M, K, device=gpu).bfloat16()
    W = (0.1 * torch.randn(K, N, device=gpu)).bfloat16()  # Conv1D weight [in, out]
    bias = torch.randn(N, device=gpu)
    acc = A.double() @ W.double()
    # bias
    out = ops.gemm(A, W, M, N, K, L.MK, L.KN, epilogue=L.EPI_BIAS, bias=bias)
    assert _rel(out, acc + bias.double()) < 1e-5
    # bias + gelu_new with the derivative side output
    dgelu = torch.empty(M, N, dtype=torch.bfloat16, device=gpu)
    act = ops.gemm(A, W, M, N, K, L.MK, L.KN, out_dtype=torch.bfloat16, epilogue=L.EPI_BIAS_GELU, bias=bias,
                   aux_out=dgelu)
    z = (acc + bias.double()).float().requires_grad_(True)
    gelu = 0.5 * z * (1.0 + torch.tanh(math.sqrt(2.0 / math.pi) * (z + 0.044715 * torch.pow(z, 3.0))))
    gelu.sum().backward()
    assert _rel(act.float(), gelu.detach()) < 6e-3
    assert _rel(dgelu.float(), z.grad) < 6e-3
    # residual add (in place)
    res = torch.randn(M, N, device=gpu)
    expect = res.double() + acc + bias.double()
    ops.gemm(A, W, M, N, K, L.MK, L.KN, out=res, epilogue=L.EPI_BIAS_RESID, bias=bias, aux=res)
    assert _rel(res, expect) < 1e-6
    # gelu backward: v * (the stored gelu')
    out = ops.gemm(A, W, M, N, K, L.MK, L.KN, out_dtype=torch.float32, epilogue=L.EPI_GELU_BWD, aux=dgelu)
    assert _rel(out, acc * dgelu.double()) < 1e-5
    # accumulate + device alpha
    base = torch.randn(M, N, device=gpu)
    alpha = torch.tensor([0.5], device=gpu)
    expect = base.double() + 0.5 * acc
    ops.gemm(A, W, M, N, K, L.MK, L.KN, out=base, epilogue=L.EPI_ACCUM, alpha_dev=alpha)
    assert _rel(base, expect) < 1e-6


def test_gemm_asymmetric_identity(gpu):
    """A = I with an asymmetric B catches a transposed C write (guide §3)."""
    n = 128
    A = torch.eye(n, device=gpu).bfloat16()
    B = torch.arange(n * n, device=gpu, dtype=torch.float32).reshape(n, n).remainder(97).bfloat16()
    for bl, Bs in ((L.KN, B), (L.NK, B.t().contiguous())):
        out = ops.gemm(A, Bs, n, n, n, L.MK, bl)
        assert torch.equal(out, B.float())


def test_gemm_rejects_bad_args(gpu):
    A = torch.randn(64, 60, device=gpu).bfloat16()
    with pytest.raises(ValueError):
        ops.gemm(A, A, 64, 64, 60, L.MK, L.NK)  # K % 8 != 0


def _attn_ref(q, k, v, causal):
    w = torch.matmul(q, k.transpose(-1, -2)) / 8.0
    if causal:
        S = q.shape[-2]
        mask = torch.tril(torch.ones(S, S, dtype=torch.bool, device=q.device))
        w = torch.where(mask, w, torch.finfo(w.dtype).min)
    p = torch.softmax(w, -1)
    return p @ v


@pytest.mark.parametrize("B,H,S,causal", [(2, 12, 128, True), (2, 12, 128, False), (1, 2, 512, True),
                                          (3, 1, 32, True), (2, 4, 100, False), (2, 2, 72, True)])
def test_attention_fwd_bwd(gpu, B, H, S, causal):
    E = 64 * H
    torch.manual_seed(B * 1000 + S + H)
    qkv = torch.randn(B * S, 3 * E, device=gpu).bfloat16()
    q, k, v = qkv[:, :E], qkv[:, E:2 * E], qkv[:, 2 * E:]
    o, lse = ops.attn_fwd(q, k, v, B, H, S, S, causal)

    def heads(t):
        return t.float().reshape(B, S, H, 64).permute(0, 2, 1, 3)
    qf, kf, vf = (heads(t).requires_grad_(True) for t in (q, k, v))
    ref = _attn_ref(qf, kf, vf, causal)
    got = o.float().reshape(B, S, H, 64).permute(0, 2, 1, 3)
    assert _rel(got, ref.detach()) < 8e-3
    w = torch.matmul(qf, kf.transpose(-1, -2)) / 8.0
    if causal:
        w = w.masked_fill(~torch.tril(torch.ones(S, S, dtype=torch.bool, device=gpu)), float("-inf"))
    assert _rel(lse, torch.logsumexp(w, -1).detach()) < 1e-4
    dout = torch.randn(B * S, E, device=gpu).bfloat16()
    ref.backward(heads(dout))
    dq, dk, dv = ops.attn_bwd(q, k, v, o, dout, lse, B, H, S, S, causal)
    for got, want in ((dq, qf.grad), (dk, kf.grad), (dv, vf.grad)):
        assert _rel(heads(got), want) < 2e-2


@pytest.mark.parametrize("B,H,Sq,Sk,causal", [(2, 12, 128, 128, True), (2, 12, 128, 128, False), (3, 2, 100, 40, False),
                                              (2, 3, 64, 128, False), (2, 2, 72, 72, True), (1, 1, 17, 17, True)])
def test_attention_bwd_short_matches_tiled(gpu, B, H, Sq, Sk, causal):
    """The one-workgroup-per-(b,h) backward (Sq, Sk <= 128) computes every product in the same order
    as the tiled dK/dV + dQ kernels: the two paths agree bit for bit."""
    E = 64 * H
    torch.manual_seed(Sq * 7 + Sk + H)
    q = torch.randn(B * Sq, E, device=gpu).bfloat16()
    kv = torch.randn(B * Sk, 2 * E, device=gpu).bfloat16()
    k, v = kv[:, :E], kv[:, E:]
    o, lse = ops.attn_fwd(q, k, v, B, H, Sq, Sk, causal)
    dout = torch.randn(B * Sq, E, device=gpu).bfloat16()
    lib = L.load()
    short = ops.attn_bwd(q, k, v, o, dout, lse, B, H, Sq, Sk, causal)
    L.check(lib.ergm_attn_tune(1), "attn_tune")
    try:
        o2, lse2 = ops.attn_fwd(q, k, v, B, H, Sq, Sk, causal)
        tiled = ops.attn_bwd(q, k, v, o, dout, lse, B, H, Sq, Sk, causal)
    finally:
        L.check(lib.ergm_attn_tune(0), "attn_tune")
    torch.cuda.synchronize()
    assert torch.equal(o, o2) and torch.equal(lse, lse2)
    for a, b in zip(short, tiled):
        assert torch.equal(a, b)


def test_attention_cross_strided(gpu):
    """Cross-attention reading K/V straight out of a stacked [T, L*2E] projection buffer."""
    B, H, S, Lyr = 2, 4, 128, 3
    E = 64 * H
    q = torch.randn(B * S, E, device=gpu).bfloat16()
    kv_all = torch.randn(B * S, Lyr * 2 * E, device=gpu).bfloat16()
    l = 1
    k = kv_all[:, l * 2 * E: l * 2 * E + E]
    v = kv_all[:, l * 2 * E + E: (l + 1) * 2 * E]
    o, lse = ops.attn_fwd(q, k, v, B, H, S, S, False)

    def heads(t):
        return t.float().reshape(B, S, H, 64).permute(0, 2, 1, 3)
    ref = _attn_ref(heads(q), heads(k), heads(v), False)
    assert _rel(heads(o), ref) < 8e-3


@pytest.mark.parametrize("B,H,Sq,Sk,causal", [(2, 3, 200, 333, False), (1, 2, 300, 300, True),
                                              (2, 2, 520, 64, False), (8, 12, 512, 512, False)])
def test_attention_tiled_ragged(gpu, B, H, Sq, Sk, causal):
    """The LDS-DMA ring kernels (Sq or Sk > 128): ragged last tiles (rows clamped, keys masked), Sq != Sk,
    K/V strided inside a wider projection buffer, the C4 cross shape; forward and backward vs fp32."""
    E = 64 * H
    torch.manual_seed(Sq * 3 + Sk + H)
    q = torch.randn(B * Sq, E, device=gpu).bfloat16()
    kv = torch.randn(B * Sk, 3 * E, device=gpu).bfloat16()  # K/V at column offsets E and 2E, ld = 3E
    k, v = kv[:, E:2 * E], kv[:, 2 * E:]
    o, lse = ops.attn_fwd(q, k, v, B, H, Sq, Sk, causal)

    def heads(t, S):
        return t.float().reshape(B, S, H, 64).permute(0, 2, 1, 3)
    qf, kf, vf = heads(q, Sq).requires_grad_(True), heads(k, Sk).requires_grad_(True), heads(v, Sk).requires_grad_(True)
    w = torch.matmul(qf, kf.transpose(-1, -2)) / 8.0
    if causal:
        w = w.masked_fill(~torch.tril(torch.ones(Sq, Sk, dtype=torch.bool, device=gpu)), float("-inf"))
    ref = torch.softmax(w, -1) @ vf
    assert _rel(heads(o, Sq), ref.detach()) < 8e-3
    assert _rel(lse, torch.logsumexp(w, -1).detach()) < 1e-4
    dout = torch.randn(B * Sq, E, device=gpu).bfloat16()
    ref.backward(heads(dout, Sq))
    dq, dk, dv = ops.attn_bwd(q, k, v, o, dout, lse, B, H, Sq, Sk, causal)
    for got, want, S in ((dq, qf.grad, Sq), (dk, kf.grad, Sk), (dv, vf.grad, Sk)):
        assert _rel(heads(got, S), want) < 2e-2


@pytest.mark.parametrize("rows,E", [(2048, 768), (100, 1024), (64, 64), (33, 128)])
def test_layernorm(gpu, rows, E):
    torch.manual_seed(rows + E)
    x = (torch.randn(rows, E, device=gpu) * 3 + 1).requires_grad_(True)
    gm = (1 + 0.1 * torch.randn(E, device=gpu)).requires_grad_(True)
    bt = (0.1 * torch.randn(E, device=gpu)).requires_grad_(True)
    y, mean, rstd = ops.layernorm_fwd(x.detach(), gm.detach(), bt.detach())
    ref = F.layer_norm(x, (E,), gm, bt, 1e-5)
    assert _rel(y.float(), ref.detach()) < 6e-3
    dy = torch.randn(rows, E, device=gpu)
    ref.backward(dy)
    dres0 = torch.randn(rows, E, device=gpu)
    dres, dres_b, dg, db = ops.layernorm_bwd(dy, x.detach(), mean, rstd, gm.detach(), dres0.clone())
    assert _rel(dres - dres0, x.grad) < 1e-5
    assert _rel(dres_b.float(), dres) < 6e-3
    assert _rel(dg, gm.grad) < 1e-5
    assert _rel(db, bt.grad) < 1e-5


@pytest.mark.parametrize("rows,cols,dt", [(2048, 768, torch.float32), (2048, 2304, torch.bfloat16),
                                          (16, 98304, torch.float32), (130, 64, torch.bfloat16)])
def test_colsum(gpu, rows, cols, dt):
    X = torch.randn(rows, cols, device=gpu).to(dt)
    out = ops.colsum(X)
    assert _rel(out, X.double().sum(0)) < 1e-6
    out2 = ops.colsum(X, out=out.clone(), accumulate=True)
    assert _rel(out2, 2 * X.double().sum(0)) < 1e-6


@pytest.mark.parametrize("B,S", [(8, 1023), (16, 1024), (32, 512), (128, 64), (96, 40)])
def test_embedding_bwd_multi_workgroup_sort(gpu, B, S):
    """3·B·S above the one-workgroup LDS sort (16384 entries): the lookups are sorted by chunked
    LDS stages + global compare-exchange passes; batches above 64 (multi-block wpe column sums).  Gradients against fp64 index_add (the sums of the
    ~B·S/2 token-type collisions per row included) and bitwise run to run."""
    E, V = 128, 50304
    g = torch.Generator().manual_seed(B * S)
    ids = torch.randint(0, 50257, (B, S), generator=g)
    ids[:, :7] = 11  # a row shared by ids and captions
    tt = torch.where(torch.arange(S) % 3 == 0, 50258, 50259).expand(B, S).contiguous()
    cap = torch.randint(0, 50257, (B, S), generator=g)
    cap[0, :9] = 11
    dh = torch.randn(B * S, E, generator=g)
    dc = torch.randn(B * S, E, generator=g)
    ref = torch.zeros(V, E, dtype=torch.float64)
    ref.index_add_(0, ids.reshape(-1), dh.double())
    ref.index_add_(0, tt.reshape(-1), dh.double())
    ref.index_add_(0, cap.reshape(-1), dc.double())
    pref = dh.double().reshape(B, S, E).sum(0)
    outs = []
    for _ in range(2):
        dwte = torch.zeros(V, E, device=gpu)
        dwpe = torch.zeros(S, E, device=gpu)
        ops.embed_bwd(ids.to(gpu), tt.to(gpu), cap.to(gpu), dh.to(gpu), dc.to(gpu), dwte, dwpe)
        outs.append((dwte, dwpe))
    dwte, dwpe = outs[0]
    assert _rel(dwte.cpu(), ref) < 1e-6
    assert _rel(dwpe.cpu(), pref) < 1e-6
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])

@pytest.mark.parametrize("with_feat", [True, False])
def test_embedding_fwd_bwd(gpu, with_feat):
    B, S, E, V = 4, 64, 256, 1000
    g = torch.Generator().manual_seed(5)
    ids = torch.randint(0, V - 3, (B, S), generator=g)
    ids[0, :10] = 7  # collisions
    tt = torch.where(torch.arange(S) < 30, V - 2, V - 1).expand(B, S).contiguous()
    cap = torch.randint(0, V - 3, (B, S), generator=g)
    cap[1, :5] = 7
    wte = torch.randn(V, E, generator=g)
    wpe = torch.randn(128, E, generator=g)
    vis = torch.randn(B, 3, E, generator=g) if with_feat else None
    aud = torch.randn(B, E, generator=g) if with_feat else None
    dev = lambda t: None if t is None else t.to(gpu)
    h0, capb = ops.embed_fwd(dev(ids), dev(tt), dev(cap), dev(wte), dev(wpe), dev(vis), dev(aud))
    wt = wte.clone().requires_grad_(True)
    wp = wpe.clone().requires_grad_(True)
    emb = F.embedding(ids, wt)
    if with_feat:
        add = torch.zeros_like(emb)
        add[:, 0] = vis[:, 0]
        add[:, 1] = aud
        emb = emb + add
    ref = emb + F.embedding(torch.arange(S), wp) + F.embedding(tt, wt)
    cref = F.embedding(cap, wt)
    assert _rel(h0.cpu(), ref.detach().reshape(B * S, E)) < 1e-7
    assert _rel(capb.float().cpu(), cref.detach().reshape(B * S, E)) < 6e-3
    dh = torch.randn(B * S, E, generator=g)
    dc = torch.randn(B * S, E, generator=g)
    (ref.reshape(B * S, E) * dh).sum().backward(retain_graph=True)
    (cref.reshape(B * S, E) * dc).sum().backward()
    base = torch.randn(V, E, generator=g)
    dwte = dev(base.clone())
    dwpe = torch.zeros(128, E, device=gpu)
    ops.embed_bwd(dev(ids), dev(tt), dev(cap), dev(dh), dev(dc), dwte, dwpe)
    assert _rel(dwte.cpu() - base, wt.grad) < 1e-6
    assert _rel(dwpe.cpu(), wp.grad) < 1e-6
    # deterministic: bitwise identical on a second run
    dwte2 = dev(base.clone())
    ops.embed_bwd(dev(ids), dev(tt), dev(cap), dev(dh), dev(dc), dwte2, dwpe)
    assert torch.equal(dwte, dwte2)


@pytest.mark.parametrize("B,S,V,ldl", [(4, 128, 50260, 50304), (2, 16, 500, 512), (3, 33, 256, 256)])
def test_cross_entropy(gpu, B, S, V, ldl):
    g = torch.Generator().manual_seed(V)
    logits = torch.zeros(B * S, ldl)
    logits[:, :V] = 3 * torch.randn(B * S, V, generator=g)
    logits[:, V:] = 1e4  # padding columns must be ignored
    lb = _bf(logits)
    labels = torch.randint(0, V, (B, S), generator=g)
    labels[:, : S // 2] = -100
    n = ops.count_valid(labels.to(gpu), V=V)[:1]
    rl, dl = ops.xent(lb.to(gpu), labels.to(gpu), n, V)
    x = lb[:, :V].float().reshape(B, S, V)[:, :-1].reshape(-1, V).requires_grad_(True)
    y = labels[:, 1:].reshape(-1)
    loss = F.cross_entropy(x, y, ignore_index=-100)
    loss.backward()
    assert int(n.item()) == int((y != -100).sum())
    assert abs(rl.sum().item() / n.item() - loss.item()) < 1e-4 * max(1.0, loss.item())
    got = dl.float().cpu().reshape(B, S, ldl)
    assert torch.all(got[:, -1] == 0) and torch.all(got[:, :, V:] == 0)
    assert _rel(got[:, :-1, :V].reshape(-1, V), x.grad) < 6e-3


@pytest.mark.parametrize("ignored", [0, 5])
def test_emotion_head(gpu, ignored):
    """CrossEntropyLoss semantics incl. ignore_index=-100 (those samples: no loss, no gradient; the mean
    is over the valid labels, src/model.py:710-711)."""
    B, S, E, Cn = 16, 8, 768, 7
    h = torch.randn(B * S, E, device=gpu).bfloat16()
    W = 0.02 * torch.randn(Cn, E, device=gpu)
    labels = torch.randint(0, Cn, (B,), device=gpu)
    labels[:ignored] = -100
    dh = torch.zeros(B * S, E, device=gpu)
    gs = torch.tensor([2.0], device=gpu)
    lm = torch.full((B, S), -100, dtype=torch.int64, device=gpu)
    counts = ops.count_valid(lm, labels, V=100, C_emo=Cn)
    assert counts.tolist() == [0, B - ignored]
    logits, loss_sum, dW = ops.emotion_head(h, W, labels, B, S, n_valid=counts[1:], dh=dh, grad_scale=gs)
    hl = h.float().reshape(B, S, E)[:, -1].clone().requires_grad_(True)
    Wr = W.clone().requires_grad_(True)
    ref = hl @ Wr.t()
    loss = F.cross_entropy(ref, labels, ignore_index=-100)
    (2.0 * loss).backward()
    assert _rel(logits, ref.detach()) < 1e-5
    assert abs(loss_sum.item() / (B - ignored) - loss.item()) < 1e-5
    assert _rel(dW, Wr.grad) < 1e-5
    assert _rel(dh.reshape(B, S, E)[:, -1], hl.grad) < 1e-5
    assert torch.all(dh.reshape(B, S, E)[:, :-1] == 0)


def test_adamw_matches_oracle(gpu):
    from oracle import gpt2_oracle as O
    n = 4096 + 64
    g = torch.Generator().manual_seed(3)
    p0 = torch.randn(n, generator=g)
    grads = [torch.randn(n, generator=g) for _ in range(3)]
    P = {"x": p0.clone()}
    st = O.AdamWState()
    p, m, v = p0.clone().to(gpu), torch.zeros(n, device=gpu), torch.zeros(n, device=gpu)
    pb = torch.empty(n, dtype=torch.bfloat16, device=gpu)
    for i, G in enumerate(grads):
        lr = O.poly_decay_lr(i, 2e-5, 1, 5) + 1e-3
        O.adamw_step(P, {"x": G}, st, lr)
        ops.adamw_step(p, G.to(gpu), m, v, pb, lr, 0.9, 0.999, 1e-8, 0.01, i + 1)
    assert torch.allclose(p.cpu(), P["x"], rtol=2e-6, atol=1e-7)
    assert torch.equal(pb.cpu(), p.cpu().bfloat16())


def test_adamw_rows_partition_equals_full_update(gpu):
    """The two row-selective passes (flag 0 rows, then flag 1 rows) are bitwise the full update; a
    capped grid (grid-stride loops) changes nothing."""
    rows, E = 300, 96
    torch.manual_seed(5)
    p0, g = torch.randn(rows * E, device=gpu), torch.randn(rows * E, device=gpu)
    m0, v0 = torch.randn(rows * E, device=gpu) * 0.1, torch.rand(rows * E, device=gpu) * 0.01
    flags = (torch.rand(rows, device=gpu) < 0.3).to(torch.uint8)
    ref = [t.clone() for t in (p0, m0, v0)]
    pb_ref = torch.empty(rows * E, dtype=torch.bfloat16, device=gpu)
    ops.adamw_step(ref[0], g, ref[1], ref[2], pb_ref, 1e-3, 0.9, 0.999, 1e-8, 0.01, 7)
    for cap in (0, 3):
        got = [t.clone() for t in (p0, m0, v0)]
        pb = torch.zeros(rows * E, dtype=torch.bfloat16, device=gpu)
        ops.adamw_rows(got[0], g, got[1], got[2], pb, E, flags, 0, 1e-3, 0.9, 0.999, 1e-8, 0.01, 7, cap)
        sel = flags.bool().repeat_interleave(E)
        assert torch.equal(got[0][sel], p0[sel])  # flagged rows untouched by the select-0 pass
        ops.adamw_rows(got[0], g, got[1], got[2], pb, E, flags, 1, 1e-3, 0.9, 0.999, 1e-8, 0.01, 7, cap)
        for a, b in zip(got, ref):
            assert torch.equal(a, b)
        assert torch.equal(pb, pb_ref)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_feature_mean_pooling(gpu, dtype):
    """ergm_feat_pool == torch.mean(last_hidden_state, dim=1) (data_process/feature_extraction.py:63,69),
    with per-sample valid lengths for padded audio, and on a strided (non-contiguous batch) view."""
    g = torch.Generator().manual_seed(5)
    img = torch.randn(4, 197, 768, generator=g).to(dtype)
    aud = torch.randn(4, 401, 768, generator=g).to(dtype)
    lens = torch.tensor([401, 250, 1, 399], dtype=torch.int32)
    v, a = ops.feat_pool(img.to(gpu)), ops.feat_pool(aud.to(gpu), lens)
    assert torch.allclose(v.cpu(), img.float().mean(1), rtol=1e-5, atol=1e-6)
    ref = torch.stack([aud[b, :int(lens[b])].float().mean(0) for b in range(4)])
    assert torch.allclose(a.cpu(), ref, rtol=1e-5, atol=1e-6)
    big = torch.randn(3, 50, 1024, generator=g).to(gpu)
    view = big[:, 10:40]  # batch stride 50*1024, frame stride 1024
    assert torch.allclose(ops.feat_pool(view).cpu(), view.float().mean(1).cpu(), rtol=1e-5, atol=1e-6)
