"""Dropout on the GPU (src/model.py:142 attention probabilities, :245 / :266 residual branches, :506
embeddings; p = 0.1 as the reference trains, src/main.py:62,129).

The masks are the build's counter-based ones (include/ergm_hip.h ergm_dropout).  Parity chain:
1. ergm_dropout_mask is bit-identical to the numpy restatement (oracle/philox.py, itself pinned by
   the Random123 known-answer vectors);
2. every fused kernel that drops (embedding forward, residual GEMM epilogue, LayerNorm backward,
   attention forward + backward) applies exactly those masks — op tests against torch with the mask;
3. the whole training step in train() mode equals the CPU oracle replaying the same masks (loss,
   logits, every gradient within the bf16 gates), at S <= 128 (one-workgroup attention backward) and
   S > 128 (tiled), with and without features;
4. eval() and p = 0 are the deterministic path, bitwise.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from ergm_amd import _lib as L
from ergm_amd import ops
from ergm_amd.config import ERGMConfig, NO_DROPOUT
from ergm_amd.model import GPT2LMHeadModel
from oracle import gpt2_oracle as O
from oracle import philox as X

pytestmark = pytest.mark.gpu
LOSS_RTOL, LOGIT_ATOL = 1e-3, 0.06


def _rel(a, b):
    a, b = torch.as_tensor(a).double().cpu(), torch.as_tensor(b).double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize("rows,cols,row0,seed,offset,site",
                         [(64, 768, 0, 1, 1, 0), (37, 61, 5, 2 ** 40 + 17, 9, 33), (192, 128, 4096, 123456789, 2, 75)])
def test_mask_generator_matches_restatement(gpu, rows, cols, row0, seed, offset, site):
    d = ops.dropout_desc(0.1, seed, offset, site, row0)
    got = ops.dropout_mask(d, rows, cols, gpu).cpu().numpy()
    want = X.keep_mask(seed, offset, site, 0.1, rows, cols, row0)
    assert np.array_equal(got, want)


def test_keep_rate_and_scale(gpu):
    p = 0.1
    d = ops.dropout_desc(p, 77, 3, 4)
    x = torch.ones(4096, 1024, device=gpu)
    ops.dropout_apply(x, d)
    vals = torch.unique(x).cpu()
    assert vals.numel() == 2 and vals[0].item() == 0.0
    assert vals[1].item() == torch.tensor(1.0 / (1.0 - p), dtype=torch.float32).item()
    rate = (x == 0).float().mean().item()
    n = x.numel()
    assert abs(rate - p) < 5 * (p * (1 - p) / n) ** 0.5
    keep = ops.dropout_mask(d, 4096, 1024, gpu)
    assert torch.equal(keep, x != 0)


def test_attention_dropout_forward_backward(gpu):
    """O = (softmax(QKᵀ/8)∘keep/(1-p))·V with the generator's mask; the stored keep bits equal it; the
    backward equals autograd through the same arithmetic (causal self and non-causal cross, S <= 128
    and the tiled S > 128 path)."""
    p = 0.1
    for (B, H, Sq, Sk, causal) in [(2, 3, 128, 128, True), (2, 2, 64, 128, False), (1, 2, 192, 192, True),
                                   (2, 1, 100, 77, False)]:
        g = torch.Generator().manual_seed(Sq + Sk)
        q = (0.5 * torch.randn(B * Sq, H * 64, generator=g)).bfloat16().to(gpu)
        k = (0.5 * torch.randn(B * Sk, H * 64, generator=g)).bfloat16().to(gpu)
        v = torch.randn(B * Sk, H * 64, generator=g).bfloat16().to(gpu)
        do = torch.randn(B * Sq, H * 64, generator=g).bfloat16().to(gpu)
        d = ops.dropout_desc(p, 99, 5, 12, row0=0)
        o, lse, bits = ops.attn_fwd(q, k, v, B, H, Sq, Sk, causal, dropout=d)
        keep = ops.dropout_mask(d, B * H * Sq, Sk, gpu)
        stored = ops.unpack_bits(bits.cpu(), Sk, 64)
        vis = torch.ones(Sq, Sk, dtype=torch.bool).tril() if causal else torch.ones(Sq, Sk, dtype=torch.bool)
        vis = vis.repeat(B * H, 1)
        assert torch.equal(stored[vis], keep.cpu()[vis])  # bits of every probability the softmax gives weight
        qf = q.float().view(B, Sq, H, 64).permute(0, 2, 1, 3).requires_grad_(True)
        kf = k.float().view(B, Sk, H, 64).permute(0, 2, 1, 3).requires_grad_(True)
        vf = v.float().view(B, Sk, H, 64).permute(0, 2, 1, 3).requires_grad_(True)
        w = qf @ kf.transpose(-1, -2) / 8.0
        if causal:
            w = w.masked_fill(~torch.ones(Sq, Sk, dtype=torch.bool, device=gpu).tril(), float("-inf"))
        pr = F.softmax(w, -1) * keep.view(B, H, Sq, Sk).float() / (1 - p)
        ref = (pr @ vf).permute(0, 2, 1, 3).reshape(B * Sq, H * 64)
        assert _rel(o.float(), ref) < 1e-2
        ref.backward(do.float())
        dq, dk, dv = ops.attn_bwd(q, k, v, o, do, lse, B, H, Sq, Sk, causal, dropout=d, keep_bits=bits)
        for got, want in ((dq, qf.grad), (dk, kf.grad), (dv, vf.grad)):
            assert _rel(got.float(), want.permute(0, 2, 1, 3).reshape(got.shape)) < 2e-2


def test_residual_dropout_epilogue_layernorm_and_embedding(gpu):
    p = 0.1
    M, N, K = 256, 768, 512
    g = torch.Generator().manual_seed(5)
    A = torch.randn(M, K, generator=g).bfloat16().to(gpu)
    W = (0.05 * torch.randn(K, N, generator=g)).bfloat16().to(gpu)
    bias = torch.randn(N, generator=g).to(gpu)
    res = torch.randn(M, N, generator=g).to(gpu)
    d = ops.dropout_desc(p, 11, 2, 7, row0=512)
    keep = ops.dropout_mask(d, M, N, gpu).float() / (1 - p)
    out = torch.empty(M, N, device=gpu)
    # C = res + drop(A·W + b)
    import ctypes as C
    dd = L.GemmDesc(M=M, N=N, K=K, lda=K, ldb=N, ldc=N, a_layout=L.MK, b_layout=L.KN, c_dtype=L.F32,
                    epilogue=L.EPI_BIAS_RESID, alpha=1.0, bias=C.c_void_p(bias.data_ptr()),
                    aux=C.c_void_p(res.data_ptr()), ld_aux=N, dropout=C.pointer(d))
    lib = L.load()
    L.check(lib.ergm_gemm(C.byref(dd), C.c_void_p(A.data_ptr()), C.c_void_p(W.data_ptr()), C.c_void_p(out.data_ptr()),
                          None, 0, C.c_void_p(torch.cuda.current_stream().cuda_stream)), "ergm_gemm")
    ref = res + (A.float() @ W.float() + bias) * keep
    assert _rel(out, ref) < 1e-4
    # LayerNorm backward: dres_bf16 = bf16(dres · keep/(1-p)), dres itself undropped
    E, rows = 768, 300
    x = torch.randn(rows, E, generator=g).to(gpu)
    gm, bt = torch.randn(E, generator=g).to(gpu), torch.randn(E, generator=g).to(gpu)
    y, mean, rstd = ops.layernorm_fwd(x, gm, bt)
    dy = torch.randn(rows, E, generator=g).to(gpu)
    dres0 = torch.randn(rows, E, generator=g).to(gpu)
    dl = ops.dropout_desc(p, 11, 3, 8)
    dres, dres_b, _, _ = ops.layernorm_bwd(dy, x, mean, rstd, gm, dres0.clone(), dropout=dl)
    dres_ref, dres_b_ref, _, _ = ops.layernorm_bwd(dy, x, mean, rstd, gm, dres0.clone())
    assert torch.equal(dres, dres_ref)
    kl = ops.dropout_mask(dl, rows, E, gpu).float() / (1 - p)
    assert torch.equal(dres_b, (dres_ref * kl).bfloat16())
    # embedding forward: h0 = drop(sum), captions untouched
    B, S, V = 2, 16, 300
    ids = torch.randint(0, V, (B, S), generator=g).to(gpu)
    tt = torch.randint(0, V, (B, S), generator=g).to(gpu)
    wte, wpe = torch.randn(V, E, generator=g).to(gpu), torch.randn(64, E, generator=g).to(gpu)
    de = ops.dropout_desc(p, 11, 4, 0, row0=32)
    h0, cap = ops.embed_fwd(ids, tt, ids, wte, wpe, dropout=de)
    h_ref, cap_ref = ops.embed_fwd(ids, tt, ids, wte, wpe)
    ke = ops.dropout_mask(de, B * S, E, gpu).float() / (1 - p)
    assert torch.equal(cap, cap_ref)
    assert torch.equal(h0, h_ref * ke)


def _masks(model, B, S, Sc=None):
    """Every keep mask of the model's last training forward, as the oracle's replay dict."""
    c = model.config
    Lr, H, E = c.n_layer, c.n_head, c.n_embd
    Sc = S if Sc is None else Sc
    seed, off = model._drop_seed, model._drop_offset
    dev = model.flat.device
    keep = {}

    def m(site, p, rows, cols):
        keep[site] = ops.dropout_mask(ops.dropout_desc(p, seed, off, site), rows, cols, dev).cpu()
    m(0, c.embd_pdrop, B * S, E)
    for l in range(Lr):
        for k in range(3):
            m(3 * l + 1 + k, c.resid_pdrop, B * S, E)
        m(3 * Lr + 1 + 2 * l, c.attn_pdrop, B * H * S, S)
        m(3 * Lr + 2 + 2 * l, c.attn_pdrop, B * H * S, Sc)
    return (c.attn_pdrop, c.resid_pdrop, c.embd_pdrop, keep)


def _grad_gate(got, ref, rtol=3e-2):
    from test_gpu_model import _grad_gate as gate
    gate(got, ref, rtol)


@pytest.mark.parametrize("B,S,feat", [(3, 64, True), (2, 128, False), (2, 192, True)])
def test_training_step_matches_oracle_mask_replay(gpu, B, S, feat):
    from ergm_amd.data import synthetic_batch
    V, E, Lr, H = 500, 128, 2, 2
    cfg = ERGMConfig(vocab_size=V, n_embd=E, n_layer=Lr, n_head=H, n_positions=256)  # p = 0.1 everywhere
    ocfg = O.OracleConfig(vocab_size=V, n_embd=E, n_layer=Lr, n_head=H, n_positions=256)
    P0 = O.init_params(ocfg, seed=41 + S)
    torch.manual_seed(S)
    model = GPT2LMHeadModel(cfg, device=gpu)
    model.load_state_dict(P0, strict=False)
    model.train()
    batch = synthetic_batch(B, S, n_turns=4, feat_dim=E, seed=42 + S, vocab_hi=V - 10, sp1=V - 2, sp2=V - 1,
                            eos=V - 4, with_features=feat)
    kw = {k: v.to(gpu) for k, v in batch.items()}
    out = model(input_ids=kw["input_ids"], token_type_ids=kw["token_type_ids"], labels=kw["labels"],
                emotion_labels=kw["emotion_labels"], caption_ids=kw["caption_ids"], imgs=kw.get("visual_feat"),
                auds=kw.get("audio_feat"))
    out.loss.backward()
    torch.cuda.synchronize()
    drop = _masks(model, B, S)
    ref, og = O.loss_and_grads(P0, ocfg, batch, dropout=drop)
    # the replay differs from the undropped oracle (the masks matter) ...
    plain, _ = O.loss_and_grads(P0, ocfg, batch)
    assert abs(plain["loss"].item() - ref["loss"].item()) > 1e-3
    # ... and the fused step equals it
    assert abs(out.loss.item() - ref["loss"].item()) <= LOSS_RTOL * abs(ref["loss"].item())
    assert (out.logits.float().cpu() - ref["logits"]).abs().max().item() <= LOGIT_ATOL
    g = {k: model.view(k, model.flat.grad).detach().float().cpu() for k in model.state_dict() if k != "lm_head.weight"}
    _grad_gate(g, og)
    # the next training forward draws fresh masks
    off = model._drop_offset
    model(**{k: v for k, v in dict(input_ids=kw["input_ids"], caption_ids=kw["caption_ids"],
                                    labels=kw["labels"]).items()}).loss.backward()
    assert model._drop_offset == off + 1


def test_eval_and_zero_p_are_the_deterministic_path(gpu):
    from ergm_amd.data import synthetic_batch
    V, E = 500, 128
    ocfg = O.OracleConfig(vocab_size=V, n_embd=E, n_layer=2, n_head=2, n_positions=64)
    P0 = O.init_params(ocfg, seed=5)
    batch = synthetic_batch(2, 64, n_turns=3, feat_dim=E, seed=6, vocab_hi=V - 10, sp1=V - 2, sp2=V - 1, eos=V - 4)
    kw = {k: v.to(gpu) for k, v in batch.items()}
    res = []
    for cfg_kw, train in ((NO_DROPOUT, True), ({}, False)):
        model = GPT2LMHeadModel(ERGMConfig(vocab_size=V, n_embd=E, n_layer=2, n_head=2, n_positions=64, **cfg_kw),
                                device=gpu)
        model.load_state_dict(P0, strict=False)
        model.train(train)
        out = model(input_ids=kw["input_ids"], token_type_ids=kw["token_type_ids"], labels=kw["labels"],
                    emotion_labels=kw["emotion_labels"], caption_ids=kw["caption_ids"], imgs=kw["visual_feat"],
                    auds=kw["audio_feat"])
        out.loss.backward()
        torch.cuda.synchronize()
        res.append((out.loss.detach().clone(), out.logits.clone(), model.flat.grad.clone()))
    for a, b in zip(*res):
        assert torch.equal(a, b)
    ref, _ = O.loss_and_grads(P0, ocfg, batch)
    assert abs(res[0][0].item() - ref["loss"].item()) <= LOSS_RTOL * abs(ref["loss"].item())
