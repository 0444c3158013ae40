"""Tensor-level wrappers over the C-ABI kernels (one HIP launch sequence per call).

Every function takes torch tensors that already live on the GPU, checks shapes/dtypes on the host,
and calls the corresponding ``ergm_*`` entry point on the current HIP stream.  No function falls back
to PyTorch or CPU: a missing library or a non-GPU tensor raises.
"""
from __future__ import annotations

import ctypes as C
import math
from typing import Optional

import torch

from . import _lib as L


def _ptr(t: Optional[torch.Tensor]):
    return None if t is None else C.c_void_p(t.data_ptr())


def _stream(dev: torch.device):
    return C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


def _need_gpu(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise ValueError("ergm_amd ops need GPU tensors (the HIP path has no CPU fallback)")


def gemm(A: torch.Tensor, B: torch.Tensor, M: int, N: int, K: int, a_layout: int = L.MK, b_layout: int = L.NK,
         out: Optional[torch.Tensor] = None, out_dtype=torch.float32, epilogue: int = L.EPI_NONE,
         bias: Optional[torch.Tensor] = None, aux: Optional[torch.Tensor] = None,
         aux_out: Optional[torch.Tensor] = None, alpha: float = 1.0, split_k: int = 0,
         alpha_dev: Optional[torch.Tensor] = None, bias_grad: Optional[torch.Tensor] = None) -> torch.Tensor:
    """C[M,N] = epilogue(alpha · A·B); A/B bf16 row-major with layouts as in ergm_hip.h.  ``bias_grad`` (f32 [N],
    KM x KN weight gradients only) also receives alpha·Σ_k B[k][n]."""
    _need_gpu(A, B)
    assert A.dtype == torch.bfloat16 and B.dtype == torch.bfloat16
    lda = A.stride(0) if A.dim() == 2 else (K if a_layout == L.MK else M)
    ldb = B.stride(0) if B.dim() == 2 else (K if b_layout == L.NK else N)
    if out is None:
        out = torch.empty(M, N, dtype=out_dtype, device=A.device)
    d = L.GemmDesc(M=M, N=N, K=K, lda=lda, ldb=ldb, ldc=out.stride(0), a_layout=a_layout, b_layout=b_layout,
                   c_dtype=L.BF16 if out.dtype == torch.bfloat16 else L.F32, epilogue=epilogue, alpha=alpha,
                   bias=_ptr(bias), aux=_ptr(aux), ld_aux=aux.stride(0) if aux is not None else 0,
                   aux_out=_ptr(aux_out), ld_aux_out=aux_out.stride(0) if aux_out is not None else 0,
                   split_k=split_k, alpha_dev=_ptr(alpha_dev), bias_grad=_ptr(bias_grad))
    lib = L.load()
    wsb = lib.ergm_gemm_workspace_size(C.byref(d))
    ws = torch.empty(max(wsb, 16), dtype=torch.uint8, device=A.device)
    L.check(lib.ergm_gemm(C.byref(d), _ptr(A), _ptr(B), _ptr(out), _ptr(ws), wsb, _stream(A.device)), "ergm_gemm")
    return out


def gemm_f8(A8: torch.Tensor, a_scale: torch.Tensor, B8t: torch.Tensor, b_scale: torch.Tensor,
            out: Optional[torch.Tensor] = None, out_dtype=torch.float32, epilogue: int = L.EPI_NONE,
            bias: Optional[torch.Tensor] = None, aux: Optional[torch.Tensor] = None,
            aux_out: Optional[torch.Tensor] = None, alpha: float = 1.0) -> torch.Tensor:
    """C[M,N] = epilogue(alpha · a_scale[m] · b_scale[n] · A8[m]·B8t[n]); A8 [M,K], B8t [N,K] e4m3 bytes
    (uint8 or torch.float8_e4m3fn), a_scale [M], b_scale [N] f32."""
    _need_gpu(A8, B8t, a_scale, b_scale)
    M, K = A8.shape
    N = B8t.shape[0]
    if out is None:
        out = torch.empty(M, N, dtype=out_dtype, device=A8.device)
    d = L.GemmDesc(M=M, N=N, K=K, lda=A8.stride(0), ldb=B8t.stride(0), ldc=out.stride(0), a_layout=L.MK,
                   b_layout=L.NK, c_dtype=L.BF16 if out.dtype == torch.bfloat16 else L.F32, epilogue=epilogue,
                   alpha=alpha, bias=_ptr(bias), aux=_ptr(aux), ld_aux=aux.stride(0) if aux is not None else 0,
                   aux_out=_ptr(aux_out), ld_aux_out=aux_out.stride(0) if aux_out is not None else 0)
    L.check(L.load().ergm_gemm_f8(C.byref(d), _ptr(A8), _ptr(a_scale), _ptr(B8t), _ptr(b_scale), _ptr(out),
                                  _stream(A8.device)), "ergm_gemm_f8")
    return out


def quant_rows_fp8(X: torch.Tensor, cols: Optional[int] = None):
    """Row-wise e4m3 quantisation: returns (Q [rows, cols] uint8, scale [rows] f32)."""
    _need_gpu(X)
    rows = X.shape[0]
    cols = X.shape[1] if cols is None else cols
    Q = torch.empty(rows, cols, dtype=torch.uint8, device=X.device)
    sc = torch.empty(rows, dtype=torch.float32, device=X.device)
    dt = L.BF16 if X.dtype == torch.bfloat16 else L.F32
    L.call("ergm_quant_rows_fp8", _ptr(X), dt, X.stride(0), rows, cols, _ptr(Q), cols, _ptr(sc), _stream(X.device))
    return Q, sc


def quant_weight_fp8(W: torch.Tensor):
    """Conv1D weight W [K, N] (f32 or bf16) → (Wt [N, K] e4m3 bytes, scale [N] f32), column-wise scales."""
    _need_gpu(W)
    K, N = W.shape
    Wt = torch.empty(N, K, dtype=torch.uint8, device=W.device)
    sc = torch.empty(N, dtype=torch.float32, device=W.device)
    ws = torch.empty(N, dtype=torch.int32, device=W.device)
    dt = L.BF16 if W.dtype == torch.bfloat16 else L.F32
    L.call("ergm_quant_weight_fp8", _ptr(W), dt, W.stride(0), K, N, _ptr(Wt), K, _ptr(sc), _ptr(ws), _stream(W.device))
    return Wt, sc


def gemm_mx(A8: torch.Tensor, a_sc: torch.Tensor, B8t: torch.Tensor, b_sc: torch.Tensor,
            out: Optional[torch.Tensor] = None, out_dtype=torch.float32, epilogue: int = L.EPI_NONE,
            bias: Optional[torch.Tensor] = None, aux: Optional[torch.Tensor] = None,
            aux_out: Optional[torch.Tensor] = None, alpha: float = 1.0, q_out: Optional[torch.Tensor] = None,
            q_sc: Optional[torch.Tensor] = None) -> torch.Tensor:
    """MX-fp8 GEMM: C[M,N] = epilogue(alpha · Σ_k dequant(A8)[m,k]·dequant(B8t)[n,k]) with A8 [M,K], B8t [N,K]
    e4m3 bytes and their e8m0 block scales (uint8, 2^(byte-127) per 32-element K block) in the library's
    K-step-major layout: a_sc [K/128, pitch >= M, 4], b_sc [K/128, pitch >= N, 4] (``mx_tile`` converts a
    [rows, K/32] array).  q_out / q_sc (BIAS_GELU / GELU_BWD): the MX copy of the bf16 output ([M,N] uint8 and
    [N/128, pitch >= M, 4])."""
    _need_gpu(A8, B8t, a_sc, b_sc)
    M, K = A8.shape
    N = B8t.shape[0]
    if out is None:
        out = torch.empty(M, N, dtype=out_dtype, device=A8.device)
    d = L.GemmDesc(M=M, N=N, K=K, lda=A8.stride(0), ldb=B8t.stride(0), ldc=out.stride(0), a_layout=L.MK,
                   b_layout=L.NK, c_dtype=L.BF16 if out.dtype == torch.bfloat16 else L.F32, epilogue=epilogue,
                   alpha=alpha, bias=_ptr(bias), aux=_ptr(aux), ld_aux=aux.stride(0) if aux is not None else 0,
                   aux_out=_ptr(aux_out), ld_aux_out=aux_out.stride(0) if aux_out is not None else 0)
    L.check(L.load().ergm_gemm_mx(C.byref(d), _ptr(A8), _ptr(a_sc), _pitch(a_sc), _ptr(B8t), _ptr(b_sc),
                                  _pitch(b_sc), _ptr(out), _ptr(q_out), _ptr(q_sc),
                                  q_out.stride(0) if q_out is not None else 0,
                                  _pitch(q_sc) if q_sc is not None else 0, _stream(A8.device)), "ergm_gemm_mx")
    return out


def _pitch(s: torch.Tensor) -> int:
    """Row pitch of an MX scale array [K/128, pitch, 4] (a 2-D [rows, 4] array: one 128-deep K step)."""
    assert s.dtype == torch.uint8 and s.is_contiguous() and s.shape[-1] == 4 and s.dim() in (2, 3)
    return s.shape[-2]


def mx_tile(S: torch.Tensor, pitch: Optional[int] = None) -> torch.Tensor:
    """[rows, nb] e8m0 block scales (block b = elements 32b..32b+31 of a row) → the library layout
    [ceil(nb/4), pitch, 4] (padding bytes 127)."""
    rows, nb = S.shape
    pitch = rows if pitch is None else pitch
    out = torch.full(((nb + 3) // 4, pitch, 4), 127, dtype=torch.uint8, device=S.device)
    Sp = torch.full((rows, out.shape[0] * 4), 127, dtype=torch.uint8, device=S.device)
    Sp[:, :nb] = S
    out[:, :rows] = Sp.reshape(rows, -1, 4).permute(1, 0, 2)
    return out


def mx_untile(T: torch.Tensor, rows: int, nb: int) -> torch.Tensor:
    """Inverse of mx_tile: [K/128, pitch, 4] → [rows, nb]."""
    return T[:, :rows].permute(1, 0, 2).reshape(rows, -1)[:, :nb].contiguous()


def quant_rows_mx(X: torch.Tensor, cols: Optional[int] = None):
    """MX-fp8 quantisation of rows: returns (Q [rows, cols] uint8 e4m3, S [ceil(cols/128), rows, 4] uint8 e8m0 in
    the library layout, ``mx_untile`` gives [rows, cols/32])."""
    _need_gpu(X)
    rows = X.shape[0]
    cols = X.shape[1] if cols is None else cols
    Q = torch.empty(rows, cols, dtype=torch.uint8, device=X.device)
    S = torch.empty((cols + 127) // 128, rows, 4, dtype=torch.uint8, device=X.device)
    dt = L.BF16 if X.dtype == torch.bfloat16 else L.F32
    L.call("ergm_quant_rows_mx", _ptr(X), dt, X.stride(0), rows, cols, _ptr(Q), cols, _ptr(S), rows,
           _stream(X.device))
    return Q, S


def quant_weight_mx(W: torch.Tensor, row_form: bool = False):
    """Conv1D weight W [K, N] (bf16) → (Wt [N, K] e4m3 bytes, S [K/128, N, 4] e8m0 block scales); with
    ``row_form`` also (Wr [K, N], Sr [N/128, K, 4]): W's rows quantised along N (the dX GEMM's B operand)."""
    _need_gpu(W)
    K, N = W.shape
    Wt = torch.empty(N, K, dtype=torch.uint8, device=W.device)
    S = torch.empty((K + 127) // 128, N, 4, dtype=torch.uint8, device=W.device)
    Wr = torch.empty(K, N, dtype=torch.uint8, device=W.device) if row_form else None
    Sr = torch.empty((N + 127) // 128, K, 4, dtype=torch.uint8, device=W.device) if row_form else None
    L.call("ergm_quant_weight_mx", _ptr(W), W.stride(0), K, N, _ptr(Wt), K, _ptr(S), N, _ptr(Wr), N, _ptr(Sr), K,
           _stream(W.device))
    return (Wt, S, Wr, Sr) if row_form else (Wt, S)


def dropout_desc(p: float, seed: int, offset: int, site: int, row0: int = 0) -> L.Dropout:
    """ergm_dropout for one site of one forward (include/ergm_hip.h)."""
    return L.Dropout(seed=seed & (2 ** 64 - 1), offset=offset & 0xFFFFFFFF, site=site, p=p, row0=row0)


def _dp(d: Optional[L.Dropout]):
    return None if d is None else C.byref(d)


def dropout_mask(d: L.Dropout, rows: int, cols: int, device) -> torch.Tensor:
    """The keep mask of dropout site ``d`` over [rows, cols] as bool (ergm_dropout_mask's bits)."""
    wpr = (cols + 31) // 32
    bits = torch.empty(rows * wpr, dtype=torch.int32, device=device)
    L.call("ergm_dropout_mask", C.byref(d), rows, cols, _ptr(bits), _stream(torch.device(device)))
    return unpack_bits(bits.view(rows, wpr), cols, 32)


def unpack_bits(words: torch.Tensor, cols: int, width: int) -> torch.Tensor:
    """[rows, n] little-endian words of `width` (32 / 64) bits -> bool [rows, cols] (bit j of word w =
    column width·w + j)."""
    rows = words.shape[0]
    b = words.contiguous().view(torch.uint8).view(rows, -1)            # little-endian bytes
    shifts = torch.arange(8, device=b.device, dtype=torch.uint8)
    bits = (b.unsqueeze(-1) >> shifts) & 1                               # [rows, bytes, 8]
    return bits.view(rows, -1)[:, :cols].bool()


def dropout_apply(x: torch.Tensor, d: L.Dropout) -> torch.Tensor:
    """In place: x = keep ? x/(1-p) : 0 (f32 [rows, cols])."""
    _need_gpu(x)
    rows, cols = x.shape
    L.call("ergm_dropout_apply", C.byref(d), _ptr(x), rows, cols, x.stride(0), _stream(x.device))
    return x


def attn_fwd(q, k, v, B, H, Sq, Sk, causal, o=None, lse=None, dropout: Optional[L.Dropout] = None):
    """q/k/v: 2-D token-major views [B*S, ld] whose first column is head 0, dim 0.  With ``dropout``
    also returns the keep bits the backward needs (u64 [B*H*Sq, ceil(Sk/64)])."""
    _need_gpu(q, k, v)
    dev = q.device
    if o is None:
        o = torch.empty(B * Sq, H * 64, dtype=torch.bfloat16, device=dev)
    if lse is None:
        lse = torch.empty(B, H, Sq, dtype=torch.float32, device=dev)
    bits = torch.zeros(B * H * Sq, (Sk + 63) // 64, dtype=torch.int64, device=dev) if dropout is not None else None
    L.call("ergm_attn_fwd", _ptr(q), _ptr(k), _ptr(v), _ptr(o), _ptr(lse), B, H, Sq, Sk, q.stride(0), k.stride(0),
           v.stride(0), o.stride(0), int(bool(causal)), _dp(dropout), _ptr(bits), _stream(dev))
    return (o, lse) if dropout is None else (o, lse, bits)


def attn_bwd(q, k, v, o, dout, lse, B, H, Sq, Sk, causal, dq=None, dk=None, dv=None,
             dropout: Optional[L.Dropout] = None, keep_bits: Optional[torch.Tensor] = None):
    _need_gpu(q, k, v, o, dout, lse)
    dev = q.device
    dq = torch.empty(B * Sq, H * 64, dtype=torch.bfloat16, device=dev) if dq is None else dq
    dk = torch.empty(B * Sk, H * 64, dtype=torch.bfloat16, device=dev) if dk is None else dk
    dv = torch.empty(B * Sk, H * 64, dtype=torch.bfloat16, device=dev) if dv is None else dv
    delta = torch.empty(B, H, Sq, dtype=torch.float32, device=dev)
    L.call("ergm_attn_bwd", _ptr(q), _ptr(k), _ptr(v), _ptr(o), _ptr(dout), _ptr(lse), _ptr(delta), _ptr(dq), _ptr(dk),
           _ptr(dv), B, H, Sq, Sk, q.stride(0), k.stride(0), v.stride(0), o.stride(0), dout.stride(0), dq.stride(0),
           dk.stride(0), dv.stride(0), int(bool(causal)), _dp(dropout), _ptr(keep_bits), _stream(dev))
    return dq, dk, dv


def layernorm_fwd(x, gamma, beta, eps=1e-5):
    _need_gpu(x, gamma, beta)
    rows, E = x.shape
    y = torch.empty(rows, E, dtype=torch.bfloat16, device=x.device)
    mean = torch.empty(rows, dtype=torch.float32, device=x.device)
    rstd = torch.empty_like(mean)
    L.call("ergm_layernorm_fwd", _ptr(x), _ptr(gamma), _ptr(beta), _ptr(y), _ptr(mean), _ptr(rstd), rows, E, eps,
           _stream(x.device))
    return y, mean, rstd


def layernorm_bwd(dy, x, mean, rstd, gamma, dres, dropout: Optional[L.Dropout] = None):
    """dres += LN_bwd(dy) in place; returns (dres, dres_bf16, dgamma, dbeta) (dres_bf16 through the
    residual-branch ``dropout`` when given)."""
    _need_gpu(dy, x, mean, rstd, gamma, dres)
    rows, E = x.shape
    lib = L.load()
    wsb = lib.ergm_layernorm_bwd_workspace_size(rows, E)
    ws = torch.empty(wsb, dtype=torch.uint8, device=x.device)
    db = torch.empty(rows, E, dtype=torch.bfloat16, device=x.device)
    dg = torch.empty(E, dtype=torch.float32, device=x.device)
    dbe = torch.empty_like(dg)
    L.call("ergm_layernorm_bwd", _ptr(dy), _ptr(x), _ptr(mean), _ptr(rstd), _ptr(gamma), _ptr(dres), _ptr(db), _ptr(dg),
           _ptr(dbe), _ptr(ws), wsb, rows, E, _dp(dropout), _stream(x.device))
    return dres, db, dg, dbe


def colsum(X, out=None, accumulate=False):
    _need_gpu(X)
    rows, cols = X.shape
    out = torch.zeros(cols, dtype=torch.float32, device=X.device) if out is None else out
    lib = L.load()
    wsb = lib.ergm_colsum_workspace_size(rows, cols)
    ws = torch.empty(max(wsb, 16), dtype=torch.uint8, device=X.device)
    L.call("ergm_colsum", _ptr(X), L.BF16 if X.dtype == torch.bfloat16 else L.F32, rows, cols, X.stride(0), _ptr(out),
           int(accumulate), _ptr(ws), wsb, _stream(X.device))
    return out


def embed_fwd(ids, tt, cap_ids, wte, wpe, vis=None, aud=None, dropout: Optional[L.Dropout] = None):
    _need_gpu(ids, cap_ids, wte, wpe)
    B, S = ids.shape
    V, E = wte.shape
    h0 = torch.empty(B * S, E, dtype=torch.float32, device=ids.device)
    cap = torch.empty(B * S, E, dtype=torch.bfloat16, device=ids.device)
    ld_vis = 0
    if vis is not None:
        vis = vis.contiguous()
        ld_vis = vis[0].numel() if vis.dim() == 3 else vis.shape[1]
    L.call("ergm_embed_fwd", _ptr(ids), _ptr(tt), _ptr(cap_ids), _ptr(wte), _ptr(wpe), _ptr(vis), ld_vis,
           _ptr(aud), _ptr(h0), _ptr(cap), B, S, E, V, _dp(dropout), _stream(ids.device))
    return h0, cap


def feat_pool(x: torch.Tensor, lengths: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None):
    """Mean over frames of encoder outputs x [B, T, D] (f32 / bf16, any row strides with unit
    last-dim stride) -> [B, D] f32; ``lengths`` [B] int32 limits each sample to its valid frames.

    The reference featurises offline (data_process/feature_extraction.py): wav2vec2-base-960h and BLIP-vision
    ``last_hidden_state`` outputs ([1, T_audio, 768] / [1, 197, 768]) mean-pooled over frames / patches
    (``torch.mean(features, dim=1)``, :63 and :69) into the 768-d vectors the model adds at positions 0 and 1
    (src/model.py:495-498).  The encoders download from the network and are out of scope; this pools encoder
    outputs already in HBM for a whole batch in one HIP kernel (``ergm_feat_pool``), padded audio included, so they
    feed the model (and at config 5 its projection GEMMs) without a host round trip."""
    _need_gpu(x)
    if x.dim() != 3 or x.stride(2) != 1:
        raise ValueError("feat_pool expects [B, T, D] with contiguous feature rows")
    B, T, D = x.shape
    if out is None:
        out = torch.empty(B, D, dtype=torch.float32, device=x.device)
    if lengths is not None:
        lengths = lengths.to(x.device, torch.int32).contiguous()
    dt = L.BF16 if x.dtype == torch.bfloat16 else L.F32
    L.call("ergm_feat_pool", _ptr(x), dt, B, T, D, x.stride(1), x.stride(0), _ptr(lengths), _ptr(out), out.stride(0),
           _stream(x.device))
    return out


def embed_bwd(ids, tt, cap_ids, dh0, dcap, dwte, dwpe):
    B, S = ids.shape
    V, E = dwte.shape
    lib = L.load()
    wsb = lib.ergm_embed_bwd_workspace_size(B * S)
    ws = torch.empty(wsb, dtype=torch.uint8, device=ids.device)
    L.call("ergm_embed_bwd", _ptr(ids), _ptr(tt), _ptr(cap_ids), _ptr(dh0), _ptr(dcap), _ptr(dwte), _ptr(dwpe),
           _ptr(ws), wsb, B, S, E, V, _stream(ids.device))


def count_valid(labels, emotion_labels=None, V: int = 2 ** 31 - 1, C_emo: int = 7):
    """int32 [2] on the device: valid LM labels (s >= 1, 0 <= y < V) and valid emotion labels."""
    B, S = labels.shape
    out = torch.empty(2, dtype=torch.int32, device=labels.device)
    L.call("ergm_count_valid", _ptr(labels), _ptr(emotion_labels), B, S, V, C_emo, _ptr(out), _stream(labels.device))
    return out


def xent(logits, labels, n_valid, V, with_grad=True):
    """logits: [B*S, ldl] bf16.  Returns (row_loss[B*S], dlogits or None)."""
    B, S = labels.shape
    rl = torch.empty(B * S, dtype=torch.float32, device=logits.device)
    dl = torch.empty_like(logits) if with_grad else None
    L.call("ergm_xent_fwd_bwd", _ptr(logits), logits.stride(0), _ptr(labels), _ptr(n_valid), _ptr(rl), _ptr(dl), B, S, V,
           1.0, _stream(logits.device))
    return rl, dl


def emotion_head(h, W, labels, B, S, n_valid=None, dh=None, grad_scale=None):
    """``n_valid``: device int32 count of valid labels (default: counted from ``labels``)."""
    E = h.shape[-1]
    Cn = W.shape[0]
    logits = torch.empty(B, Cn, dtype=torch.float32, device=h.device)
    loss_sum = torch.empty(1, dtype=torch.float32, device=h.device)
    dW = torch.empty_like(W) if dh is not None else None
    scratch = torch.empty(B * (Cn + 1), dtype=torch.float32, device=h.device)
    if labels is not None and n_valid is None:
        n_valid = ((labels >= 0) & (labels < Cn)).sum().to(torch.int32).reshape(1)
    L.call("ergm_emotion_head", _ptr(h), _ptr(W), _ptr(labels), _ptr(logits), _ptr(loss_sum), _ptr(dW), _ptr(dh),
           _ptr(scratch), B, S, E, Cn, _ptr(n_valid), _ptr(grad_scale), _stream(h.device))
    return logits, loss_sum, dW


def adamw_step(p, g, m, v, p_bf16, lr, beta1, beta2, eps, weight_decay, step, max_blocks=0):
    """One torch.optim.AdamW step (flat fp32 buffers), bias corrections formed in double like torch.
    ``max_blocks`` > 0 caps the grid (for updates overlapped with other work)."""
    import math
    bc1 = 1 - beta1 ** step
    bc2 = 1 - beta2 ** step
    L.call("ergm_adamw_step", _ptr(p), _ptr(g), _ptr(m), _ptr(v), _ptr(p_bf16), p.numel(), lr, beta1, beta2, eps,
           weight_decay, lr / bc1, math.sqrt(bc2), int(max_blocks), _stream(p.device))


def adamw_rows(p, g, m, v, p_bf16, row_len, row_flag, select, lr, beta1, beta2, eps, weight_decay, step,
               max_blocks=0):
    """``adamw_step`` restricted to rows r of the [numel/row_len, row_len] block with
    (row_flag[r] != 0) == select (row_flag: a uint8 tensor or a raw device pointer)."""
    import math
    bc1 = 1 - beta1 ** step
    bc2 = 1 - beta2 ** step
    rows = p.numel() // row_len
    flag = C.c_void_p(row_flag) if isinstance(row_flag, int) else _ptr(row_flag)
    L.call("ergm_adamw_rows", _ptr(p), _ptr(g), _ptr(m), _ptr(v), _ptr(p_bf16), rows, row_len, flag, int(select), lr,
           beta1, beta2, eps, weight_decay, lr / bc1, math.sqrt(bc2), int(max_blocks), _stream(p.device))


def cast_bf16(src, dst):
    L.call("ergm_cast_bf16", _ptr(src), _ptr(dst), src.numel(), _stream(src.device))


def axpy(x, y, alpha=1.0):
    L.call("ergm_axpy", _ptr(x), _ptr(y), x.numel(), alpha, _stream(x.device))
