/*
 * ergm_hip.h — C-ABI of libergm_hip.so, the MI355X (gfx950) implementation of ERGM's fused GPT-2
 * training step (LovesickPatience/ERGM src/model.py + the src/main.py train step).
 *
 * Every entry point is `extern "C"`, takes plain pointers + sizes + an explicit hipStream_t
 * (passed as void*), never allocates on the hot path (the caller passes workspace), never frees or
 * retains caller memory, and returns 0 (ERGM_OK) or a negative ergm_status.  A thread-local
 * message is kept for the last error (ergm_last_error).  All calls are asynchronous on `stream`,
 * re-entrant and callable from any host thread (PyTorch's autograd worker thread included).
 *
 * Which reference interface each entry replaces (paths relative to /root/reference):
 *   ergm_gemm             transformers Conv1D.forward (addmm, W stored [in,out]) used at
 *                         src/model.py:95-99,257-258 and its autograd backward (dX = dY·Wᵀ,
 *                         dW = Xᵀ·dY); nn.Linear lm_head (src/model.py:605,698)
 *   ergm_attn_fwd         GPT2Attention._attn src/model.py:119-148 (+ _split_heads/_merge_heads
 *                         :190-198 folded into addressing)
 *   ergm_attn_bwd         autograd backward of the same
 *   ergm_layernorm_fwd    nn.LayerNorm (src/model.py:276,278,282,392; applied :298,318,332,578)
 *   ergm_layernorm_bwd    its autograd backward
 *   ergm_embed_fwd        wte/wpe lookups + visual/audio injection + token-type add
 *                         (src/model.py:459-463,495-504)
 *   ergm_embed_bwd        Embedding backward into the tied wte / wpe
 *   ergm_xent_fwd_bwd     CrossEntropyLoss(ignore_index=-100) on shifted logits (src/model.py:704-708)
 *   ergm_emotion_head     emotion_head + its CrossEntropyLoss (src/model.py:700-701,710-711)
 *   ergm_adamw_step       torch.optim.AdamW.step (src/main.py:68,155)
 *   ergm_model_*          the whole GPT2LMHeadModel.forward (src/model.py:654-737) and its
 *                         backward (src/main.py:154) as one native launch sequence
 */
#ifndef ERGM_HIP_H
#define ERGM_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ERGM_ABI_VERSION 11  /* 11: ergm_dp_sum_adamw takes max_blocks */

typedef enum {
    ERGM_OK = 0,
    ERGM_EINVAL = -1,        /* bad shape / stride / dtype / alignment / null pointer */
    ERGM_EUNSUPPORTED = -2,  /* valid request this build does not implement */
    ERGM_EHIP = -3,          /* HIP launch / runtime failure (hipError_t in the message) */
} ergm_status;

/* Dropout (nn.Dropout of the reference model in training mode: attention probabilities
 * src/model.py:142, attention / cross-attention resid_dropout :245, MLP dropout :266, embedding
 * dropout :506; p = GPT2Config attn_pdrop / resid_pdrop / embd_pdrop, 0.1 for the "gpt2" checkpoint
 * src/main.py:62).  The keep decision of element (row, col) of a dropout site is a pure function of
 * (seed, offset, site, row0 + row, col): Philox4x32-10 with key = seed and counter =
 * {g mod 2^32, g >> 32, site, offset}, g = (row0 + row)·ceil(cols/4) + col/4; the element takes word
 * (col mod 4) and is dropped iff that word < round(p·2^32); kept elements are scaled by 1/(1-p).
 * Backward passes recompute the elementwise sites' bits; the attention forward stores its keep bits
 * (1 bit per probability, ergm_attn_fwd) for the backward.  For the elementwise sites rows are
 * tokens (b·S + s) and cols = n_embd; for attention probabilities rows are (b·H + h)·Sq + q and
 * cols = Sk.  p = 0 or a NULL descriptor: no dropout.                                               */
typedef struct {
    uint64_t seed;
    uint32_t offset;   /* forward number: every training forward draws fresh masks */
    uint32_t site;     /* which nn.Dropout: ergm_drop_site */
    float p;           /* drop probability, [0, 1) */
    int64_t row0;      /* global row of the caller's row 0 (data-parallel ranks, batch slices) */
} ergm_dropout;

/* Site numbering of the executor (L blocks): 0 = embedding dropout; 3l+1 / 3l+2 / 3l+3 = the
 * attention / cross-attention / MLP residual-branch dropout of block l (the residual-stream tensor
 * they produce); 3L+1+2l / 3L+2+2l = attention / cross-attention probabilities of block l. */
#define ERGM_DROP_SITE_EMBD 0u
#define ERGM_DROP_SITE_RESID(l, k) (3u * (uint32_t)(l) + 1u + (uint32_t)(k)) /* k: 0 attn, 1 cross, 2 mlp */
#define ERGM_DROP_SITE_ATTN(L, l, cross) (3u * (uint32_t)(L) + 1u + 2u * (uint32_t)(l) + ((cross) ? 1u : 0u))

/* The keep mask itself: bits[r][w], ceil(cols/32) words per row, bit j of word w = element
 * (r, 32w + j) kept (pad bits 0).  Tests replay these masks through the CPU oracle.               */
int ergm_dropout_mask(const ergm_dropout* d, int rows, int cols, uint32_t* bits, void* stream);
/* x[r][c] = keep ? x·1/(1-p) : 0, in place (f32, row stride ld; cols, ld multiples of 4). */
int ergm_dropout_apply(const ergm_dropout* d, float* x, int rows, int cols, int ld, void* stream);

typedef enum { ERGM_F32 = 0, ERGM_BF16 = 1 } ergm_dtype;

/* Operand storage layouts (row-major storage, leading dimension in elements).
 *   A: ERGM_MK = A[m][k] (k contiguous)   ERGM_KM = A[k][m] (m contiguous)
 *   B: ERGM_NK = B[n][k] (nn.Linear weight, k contiguous)
 *      ERGM_KN = B[k][n] (Conv1D weight [in,out], n contiguous)                    */
typedef enum { ERGM_MK = 0, ERGM_KM = 1 } ergm_a_layout;
typedef enum { ERGM_NK = 0, ERGM_KN = 1 } ergm_b_layout;

/* Epilogues applied to v = alpha * (A·B)[m][n] (all math fp32):
 *   NONE        C = v
 *   BIAS        C = v + bias[n]
 *   BIAS_GELU   C = gelu_new(v + bias[n]); aux_out[m][n] = bf16(gelu_new'(v + bias[n])) (the
 *               derivative the backward multiplies by)
 *   BIAS_RESID  C(f32) = aux[m][n](f32) + drop(v + bias[n])      (residual add; aux may == C;
 *               drop = the optional `dropout` site over [M][N], identity when NULL)
 *   GELU_BWD    C = v * aux[m][n] with aux = the bf16 gelu_new' that BIAS_GELU stored
 *   ACCUM       C(f32) = C + v                                   (beta = 1 accumulation)          */
typedef enum {
    ERGM_EPI_NONE = 0,
    ERGM_EPI_BIAS = 1,
    ERGM_EPI_BIAS_GELU = 2,
    ERGM_EPI_BIAS_RESID = 3,
    ERGM_EPI_GELU_BWD = 4,
    ERGM_EPI_ACCUM = 5,
} ergm_epilogue;

typedef struct {
    int M, N, K;
    int lda, ldb, ldc;
    int a_layout;   /* ergm_a_layout */
    int b_layout;   /* ergm_b_layout */
    int c_dtype;    /* ergm_dtype of C (A and B are bf16) */
    int epilogue;   /* ergm_epilogue */
    float alpha;
    const float* bias;   /* [N] f32 or NULL */
    const void* aux;     /* epilogue input: f32 residual [M][ld_aux] or bf16 gelu' */
    int ld_aux;
    void* aux_out;       /* epilogue second output (bf16 gelu' of the pre-activation) [M][ld_aux_out] */
    int ld_aux_out;
    int split_k;         /* 0 = choose automatically, 1 = none, >1 = forced split count */
    const float* alpha_dev;  /* optional device scalar multiplied into alpha (autograd grad_output) */
    const ergm_dropout* dropout;  /* BIAS_RESID only: residual-branch dropout (rows m, cols n); NULL = none */
    float* bias_grad;    /* a_layout KM + b_layout KN (a weight gradient Xᵀ·dY), epilogue NONE, f32 C only:
                          * also write alpha·Σ_k B[k][n] (the Conv1D bias gradient, column sums of dY over
                          * the K tokens) to bias_grad[n], f32 [N]; NULL = none.  Computed from the B
                          * fragments the GEMM already stages (no second pass over dY), deterministic. */
} ergm_gemm_desc;

/* Tuning hook (calling thread only): force pipelined-kernel configuration `cfg` (tile / wave grid /
 * LDS stages, see kCfgs in ergm_amd/csrc/gemm.hip) and split-K count for later ergm_gemm calls;
 * cfg = -1 restores the automatic choice.  Used by tools/gemm_tune.py.                          */
int ergm_gemm_tune(int cfg, int split);
/* Per-shape override of the automatic choice: GEMMs of exactly (M, N, K, a_layout, b_layout) with
 * split_k == 0 use configuration `cfg` and `split`; cfg = -1 removes the entry.  Process-wide, set
 * before the plans that use it are created (their workspace is sized then).  ergm_gemm_trace(on,
 * shapes, max) records the distinct shapes of later ergm_gemm calls (on = 1 starts a new record) and
 * returns how many were recorded so far, copying up to `max` of them as 5 ints (M, N, K, layouts).
 * Both serve tools/step_tune.py, which measures configurations inside the running training step. */
int ergm_gemm_set_override(int M, int N, int K, int a_layout, int b_layout, int cfg, int split);
int ergm_gemm_trace(int on, int* shapes, int max_shapes);
/* Workspace bytes ergm_gemm needs for `desc` (split-K partial slabs); 0 if none. */
size_t ergm_gemm_workspace_size(const ergm_gemm_desc* desc);
int ergm_gemm(const ergm_gemm_desc* desc, const void* A, const void* B, void* C, void* workspace,
              size_t ws_bytes, void* stream);

/* fp8 GEMM (config 5's forward Conv1D GEMMs; build-side, the reference is fp32):
 *   C = epilogue(alpha · a_scale[m] · b_scale[n] · Σ_k A[m][k]·B[n][k])
 * A [M][lda], B [N][ldb]: OCP e4m3fn bytes, k contiguous (desc->a_layout = ERGM_MK, b_layout =
 * ERGM_NK); K % 128 == 0; lda, ldb multiples of 16.  Runs v_mfma_scale_f32_16x16x128_f8f6f4 (unit
 * block scales; 2x the bf16 MFMA rate).  Epilogues: NONE (f32/bf16 C), BIAS / BIAS_GELU (bf16 C),
 * BIAS_RESID (f32 C).  ergm_gemm_f8_tune forces a tile configuration (-1 = automatic).           */
int ergm_gemm_f8(const ergm_gemm_desc* desc, const void* A, const float* a_scale, const void* B,
                 const float* b_scale, void* C, void* stream);
int ergm_gemm_f8_tune(int cfg);
/* Per-shape tile configuration of the fp8 / MX GEMMs (ergm_gemm_f8, ergm_gemm_mx) keyed on (M, N, K): the in-step
 * tuner's hook (tools/step_tune.py --f8), as ergm_gemm_set_override is for the bf16 GEMMs; cfg -1 removes the entry.
 * ergm_gemm_trace lists these GEMMs with a_layout 16.  ABI 10. */
int ergm_gemm_f8_set_override(int M, int N, int K, int cfg);
/* Row-wise e4m3 quantisation (activations): scale[r] = max_c |X[r][c]| / 448 (1 for a zero row),
 * Q[r][c] = e4m3(clamp(X[r][c] / scale[r], ±448)).  X bf16 or f32 (x_dtype), cols % 8 == 0.       */
int ergm_quant_rows_fp8(const void* X, int x_dtype, int ldx, int rows, int cols, void* Q, int ldq,
                        float* scale, void* stream);
/* Column-wise e4m3 quantisation of a Conv1D weight W [K][ldw] (in, out; f32 or bf16 per w_dtype)
 * into its transpose Wt [N][ldt] (k contiguous, the B operand of ergm_gemm_f8): scale[n] =
 * max_k |W[k][n]| / 448.  amax_ws: N x 4 bytes of workspace.  K, N multiples of 64.             */
int ergm_quant_weight_fp8(const void* W, int w_dtype, int ldw, int K, int N, void* Wt, int ldt,
                          float* scale, void* amax_ws, void* stream);

/* MX-fp8 (OCP microscaling) GEMM, config 5's forward: A [M][lda]
 * and B [N][ldb] e4m3fn bytes (k contiguous),
 * each with an e8m0 scale byte per 32-element K block (a_scale [M][ld_sa], b_scale [N][ld_sb]: 2^(byte-127)),
 *   C = epilogue(alpha · Σ_blocks 2^(ea+eb-254) · Σ_{k in block} A[m][k]·B[n][k])
 * on v_mfma_scale_f32_16x16x128_f8f6f4 with the block scales consumed by the MFMA (no dequantisation pass).
 * Scale layout (every MX scale array of this library): the 4 bytes of one row's 128-deep K step form a word and
 * the words of one K step are contiguous over the rows — byte (row r, block b) at ((b/4)·pitch + r)·4 + b%4, with
 * pitch >= the row count (ld_sa >= M, ld_sb >= N, ld_qs >= M), so a GEMM stage loads its scales as whole lines.
 * K % 128 == 0.  Epilogues as ergm_gemm_f8, plus GELU_BWD (bf16 C,
 * aux = gelu_new').  q_out / q_scale (BIAS_GELU or GELU_BWD, N % 32 == 0): the epilogue also writes the MX copy
 * of its bf16 output, [M][ld_q] e4m3 and
 * [M][ld_qs] e8m0 (the next MX GEMM's A operand).  Tile configurations as ergm_gemm_f8 (ergm_gemm_f8_tune). */
int ergm_gemm_mx(const ergm_gemm_desc* desc, const void* A, const void* a_scale, int ld_sa, const void* B,
                 const void* b_scale, int ld_sb, void* C, void* q_out, void* q_scale, int ld_q, int ld_qs, void* stream);
/* MX-fp8 quantisation of rows (activations): block b of row r = columns 32b..32b+31; e = the smallest integer
 * with max|block| <= 448·2^e (0 for a zero block), scale byte (r, b) = e + 127 in the layout above (pitch lds >=
 * rows), Q[r][c] = e4m3(X[r][c]·2^-e) (exact scaling, round to nearest even, never saturating).  X bf16 or f32
 * (x_dtype), cols % 32 == 0.                                                                                  */
int ergm_quant_rows_mx(const void* X, int x_dtype, int ldx, int rows, int cols, void* Q, int ldq, void* S, int lds,
                       void* stream);
/* MX-fp8 quantisation of a Conv1D weight W [K][ldw] (bf16) into its transpose Wt [N][ldt] (k contiguous) with a
 * scale per (column n, 32-row block): S, pitch lds >= N; same rule as ergm_quant_rows_mx; one pass, no amax pass.
 * Optionally (Wr != NULL) in the same pass the row form — Wr [K][ldr] e4m3 with a scale per (row k, 32-column
 * block), Sr pitch ldsr >= K: the B operand of the data-gradient GEMM dX = dY·Wᵀ.  K, N multiples of 64.       */
int ergm_quant_weight_mx(const void* W, int ldw, int K, int N, void* Wt, int ldt, void* S, int lds, void* Wr, int ldr,
                         void* Sr, int ldsr, void* stream);

/* Fused attention over head_dim = 64, token-major tensors with head h at columns [64h, 64h+64):
 *   Q[b][s][h*64+d] = q + (b*Sq + s)*ldq + h*64 + d     (likewise K/V with Sk rows, O with ldo)
 * out: O (bf16) and lse[b][h][s] = ln Σ_k exp(score) (f32; backward recomputes P from it).
 * `causal`: key j visible to query i iff j <= i (Sq == Sk required). scale = 1/sqrt(64).
 * dropout (optional, p > 0): O = (P∘keep/(1-p))·V with the keep bits of ergm_dropout_mask over rows
 * (b·H + h)·Sq + q and cols Sk (the LSE stays that of the undropped softmax); the forward stores them
 * in keep_bits: u64 [B·H·Sq][ceil(Sk/64)], bit key mod 64 of word key/64 (Sq, Sk <= 1024); the
 * backward reads the same buffer.  NULL / p == 0: no dropout, keep_bits unused.                  */
int ergm_attn_fwd(const void* q, const void* k, const void* v, void* o, float* lse, int B, int H,
                  int Sq, int Sk, int ldq, int ldk, int ldv, int ldo, int causal,
                  const ergm_dropout* dropout, void* keep_bits, void* stream);
/* delta workspace: B*H*Sq floats.  dq/dk/dv are bf16 with their own leading dims.              */
int ergm_attn_bwd(const void* q, const void* k, const void* v, const void* o, const void* dout,
                  const float* lse, float* delta, void* dq, void* dk, void* dv, int B, int H, int Sq,
                  int Sk, int ldq, int ldk, int ldv, int ldo, int lddo, int lddq, int lddk, int lddv,
                  int causal, const ergm_dropout* dropout, const void* keep_bits, void* stream);
/* Path selection hook (tests / tuning): bit 0 of force_generic makes ergm_attn_bwd use the tiled
 * kernels even where the one-workgroup-per-(b,h) kernel applies (Sq, Sk <= 128; the forward is tiled at
 * every length); bits 4-7 select the
 * tiled kernels' LDS ring depth (0 = per-kernel defaults; 2, 3 or 4).  Process-wide; not for concurrent use with
 * running attention calls. */
int ergm_attn_tune(int force_generic);

/* LayerNorm over rows of E (biased variance, eps): y(bf16) = (x-μ)·rstd·γ + β; x f32.        */
int ergm_layernorm_fwd(const float* x, const float* gamma, const float* beta, void* y, float* mean,
                       float* rstd, int rows, int E, float eps, void* stream);
/* dres(f32, in/out) += LN_bwd(dy); dres_bf16 (optional) = bf16(dres), or bf16(dres·keep/(1-p))
 * with `dropout` (rows x E): the gradient of the residual branch whose dropped output was added into
 * this residual-stream tensor; dγ/dβ (f32 [E], written).
 * workspace: ergm_layernorm_bwd_workspace_size(rows, E) bytes.                                  */
size_t ergm_layernorm_bwd_workspace_size(int rows, int E);
int ergm_layernorm_bwd(const float* dy, const float* x, const float* mean, const float* rstd,
                       const float* gamma, float* dres, void* dres_bf16, float* dgamma, float* dbeta,
                       void* workspace, size_t ws_bytes, int rows, int E, const ergm_dropout* dropout,
                       void* stream);

/* Column sums of a row-major matrix (bias gradients, wpe gradient): out[c] (=|+=) Σ_r X[r][c]. */
size_t ergm_colsum_workspace_size(int rows, int cols);
int ergm_colsum(const void* X, int x_dtype, int rows, int cols, int ldx, float* out, int accumulate,
                void* workspace, size_t ws_bytes, void* stream);

/* Embedding + fusion (src/model.py:459-463,495-506):
 *   h0[b,s] = drop(((wte[ids] + [s==0]·vis[b] + [s==1]·aud[b]) + wpe[s]) + wte[tt])      (f32)
 *   cap[b,s] = bf16(wte[cap_ids])                       (caption embeddings are not dropped)
 * vis: [B][ld_vis] row b's first E values (imgs[i][0]); vis/aud may be NULL (text-only);
 * tt may be NULL; dropout (rows b·S + s, cols E) may be NULL.                                  */
int ergm_embed_fwd(const int64_t* ids, const int64_t* tt, const int64_t* cap_ids, const float* wte,
                   const float* wpe, const float* vis, int ld_vis, const float* aud, float* h0,
                   void* cap, int B, int S, int E, int V, const ergm_dropout* dropout, void* stream);
/* Feature pooling (data_process/feature_extraction.py:63,69: torch.mean(last_hidden_state, dim=1) of the
 * wav2vec2 / BLIP-vision encoder outputs): out[b][d] = mean_{t < len_b} x[b][t][d], x f32 or bf16 with
 * strides ld_t (frames) and ld_b (samples) in elements, lengths optional (NULL = all T frames; padded
 * audio otherwise), out f32 [B][ld_out].  Fixed summation order (deterministic).                   */
int ergm_feat_pool(const void* x, int x_dtype, int B, int T, int D, long ld_t, long ld_b,
                   const int* lengths, float* out, int ld_out, void* stream);
/* Deterministic (sorted segment-sum) embedding backward:
 *   dwte[v] += Σ_{t: ids[t]=v} dh0[t] + Σ_{t: tt[t]=v} dh0[t] + Σ_{t: cap[t]=v} dcap[t]
 *   dwpe[s]  = Σ_b dh0[b,s]
 * workspace: ergm_embed_bwd_workspace_size(B*S) bytes.                                          */
size_t ergm_embed_bwd_workspace_size(int T);
int ergm_embed_bwd(const int64_t* ids, const int64_t* tt, const int64_t* cap_ids, const float* dh0,
                   const float* dcap, float* dwte, float* dwpe, void* workspace, size_t ws_bytes,
                   int B, int S, int E, int V, void* stream);

/* Shifted LM cross-entropy, fused forward+backward over bf16 logits [B*S][ldl] (columns >= V
 * ignored, zeroed in dlogits).  Row t=(b,s) is valid iff s < S-1 and labels[b][s+1] != -100.
 * n_valid_global: device int (count of valid rows over all DP ranks).
 * row_loss[t] = lse - logit[target] (0 for invalid); dlogits = grad_scale·(softmax - onehot)/n_valid
 * (bf16, may be NULL for forward only).  ergm_count_valid writes the local counts: counts[0] = LM
 * labels at s >= 1 with 0 <= y < V, counts[1] = emotion labels with 0 <= y < C (either label tensor
 * may be NULL: count 0).  Labels outside the range (-100 = torch's ignore_index) are ignored.       */
int ergm_count_valid(const int64_t* labels, const int64_t* emotion_labels, int B, int S, int V, int C,
                     int* counts, void* stream);
int ergm_xent_fwd_bwd(const void* logits, int ldl, const int64_t* labels, const int* n_valid_global,
                      float* row_loss, void* dlogits, int B, int S, int V, float grad_scale,
                      void* stream);
/* Emotion head on the last token: logits[b][c] = Σ_e h[b,S-1,e]·W[c][e] (h bf16, W f32 [C][E]);
 * with labels: loss_sum = Σ_b CE_b over valid labels (0 <= y < C; others, e.g. -100, are ignored),
 * scratch = B*(C+1) floats, n_valid_global = device count of valid labels (all DP ranks); with dW/dh:
 * dW[C][E] written and dh[b,S-1,:] += dlogits·W (f32 dh [B*S][E]), dlogits =
 * (softmax - onehot)·grad_scale/n_valid (0 for ignored labels).                                  */
int ergm_emotion_head(const void* h, const float* W, const int64_t* labels, float* logits,
                      float* loss_sum, float* dW, float* dh, float* scratch, int B, int S, int E, int C,
                      const int* n_valid_global, const float* grad_scale_dev, void* stream);
/* out[0] = Σ row_loss / n_valid_global (0 if n_valid_global is NULL), out[1] = emo_loss_sum /
 * n_valid_emo (0 if emo_loss_sum is NULL), out[2] = out[0]+out[1]; a zero count gives 0/0 = NaN,
 * as torch's mean CrossEntropyLoss does.                                                         */
int ergm_loss_finalize(const float* row_loss, int T, const int* n_valid_global,
                       const float* emo_loss_sum, const int* n_valid_emo, float* out, void* stream);

/* torch.optim.AdamW step over flat fp32 arrays; also refreshes the bf16 shadow copy.
 * Arithmetic in torch's order: p*=(1-lr·wd); m=lerp(m,g,1-β1); v=β2·v+(1-β2)g²;
 * p -= step_size · m / (sqrt(v)/bc2_sqrt + eps), step_size = lr/(1-β1^t), bc2_sqrt = sqrt(1-β2^t).
 * lr, β1, β2 and weight_decay are doubles (ABI 5): torch forms 1-lr·wd, 1-β1 and 1-β2 from the Python
 * doubles and rounds each once to fp32 (from a float β2 = 0.999f, 1-β2 is off by 1.3e-5 relative).
 * max_blocks > 0 caps the grid (grid-stride loop): an update running concurrently with the backward
 * on another stream then occupies only that many CUs instead of flooding the chip; 0 = full grid. */
int ergm_adamw_step(float* p, const float* g, float* m, float* v, void* p_bf16, size_t n, double lr,
                    double beta1, double beta2, float eps, double weight_decay, float step_size,
                    float bc2_sqrt, int max_blocks, void* stream);
/* The same update restricted to the rows of a [rows][row_len] block whose flag byte matches:
 * row r is updated iff (row_flag[r] != 0) == (select != 0).  With ergm_model_set_row_flags this
 * splits the tied-embedding update into the rows only the LM head touched (final early in the
 * backward) and the rows the lookups touched (final after the embedding backward). */
int ergm_adamw_rows(float* p, const float* g, float* m, float* v, void* p_bf16, int rows, int row_len,
                    const void* row_flag, int select, double lr, double beta1, double beta2, float eps,
                    double weight_decay, float step_size, float bc2_sqrt, int max_blocks, void* stream);
/* bf16 shadow copy of fp32 values: dst[i] = bf16(src[i]). */
int ergm_cast_bf16(const float* src, void* dst, size_t n, void* stream);
/* y[i] += x[i] (f32), used to accumulate gradients across backward calls. */
int ergm_axpy(const float* x, float* y, size_t n, float alpha, void* stream);
/* Data-parallel gradient exchange in bf16 with fp32 accumulation (ergm_amd/dist.py): after an
 * all-to-all of bf16 gradient chunks, out[i] = bf16(Σ_{j < nchunks} in[j·chunk + i]) summed in fp32
 * in rank order j; after the all-gather, dst[i] = f32(src[i]).  chunk, n multiples of 4.           */
int ergm_chunk_sum_bf16(const void* in, int nchunks, size_t chunk, void* out, void* stream);
/* ZeRO-1 reduce-scatter tail: the same rank-order fp32 sum of the nchunks copies, rounded once to bf16 and
 * written widened to fp32 (out[i], i < n <= chunk, n % 4 == 0): this rank's reduced gradient chunk. */
int ergm_chunk_sum_bf16_f32(const void* in, int nchunks, size_t chunk, size_t n, float* out, void* stream);
/* Data-parallel bucket helpers (ergm_amd/dist.py, ZeRO-1 bf16 exchange), one launch each where the Python path
 * issued two or three: ergm_dp_pack_bf16 casts a bucket's n fp32 gradients into the all-to-all send buffer and zeroes
 * its padding up to `total`; ergm_dp_sum_adamw sums the received chunks in rank order, rounds once to bf16 (the
 * ergm_chunk_sum_bf16_f32 value, bitwise), writes the widened sum into grad[0..n) and applies ergm_adamw_step's
 * update to p / m / v [0..n) with it, the updated bf16 parameters going to `shadow` (this rank's all-gather slot);
 * max_blocks > 0 caps its grid like ergm_adamw_step's (an update overlapped with the backward's GEMMs). */
int ergm_dp_pack_bf16(const float* src, size_t n, void* dst, size_t total, void* stream);
int ergm_dp_sum_adamw(const void* in, int nchunks, size_t chunk, size_t n, float* grad, float* p, float* m, float* v,
                      void* shadow, double lr, double beta1, double beta2, float eps, double weight_decay,
                      float step_size, float bc2_sqrt, int max_blocks, void* stream);
int ergm_cast_f32(const void* src, float* dst, size_t n, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Whole-model executor.  The caller owns every buffer; ergm_model_plan only records pointers and
 * dimensions (see ergm_amd/model.py for the layout it builds).  Forward = src/model.py:654-737;
 * backward = loss.backward() (src/main.py:154), with per-layer entry points so a data-parallel
 * caller can start gradient all-reduce buckets as layers finish.
 * ------------------------------------------------------------------------------------------- */
typedef struct ergm_model_plan ergm_model_plan;

typedef struct {
    int vocab, vocab_pad, n_embd, n_layer, n_head, n_inner, n_positions;
    int batch, seq;           /* local (per-rank) batch and sequence length */
    float eps;
    int has_features;         /* visual/audio injection present */
    int ld_vis;               /* row stride of the visual feature (Tv*Fd when [B,Tv,Fd]) */
    int feat_dim;             /* Fd: width of the pooled features; 0 or n_embd = added directly
                               * (src/model.py:497-498); otherwise a Conv1D projection per modality
                               * (build-side, config 5: 768-d features into a 1024-d backbone) */
    int fp8;                  /* 1: the forward Conv1D GEMMs of every block (and the caption K/V
                               * GEMM) run on fp8: ergm_gemm_mx on MX-fp8 operands (default; the
                               * LayerNorms, the GELU epilogue and the attention forward write the MX
                               * copies of their outputs) or, with ERGM_FP8_MX=0, ergm_gemm_f8 with
                               * per-row activation / per-column weight scales; weights are
                               * re-quantised from the bf16 shadow at every forward; LM head,
                               * backward and optimizer stay bf16/f32 */
} ergm_model_dims;

/* Pointer table: names follow the reference state_dict; see ergm_amd/model.py. */
typedef struct {
    /* fp32 master params and their bf16 shadows (same element offsets) */
    const float* wte;  const void* wte_b;   /* [vocab_pad][E] */
    const float* wpe;                        /* [n_positions][E] */
    const float* ln_f_w; const float* ln_f_b;
    const float* emo_w;                      /* [7][E] */
    const void* capkv_w_b; const float* capkv_b;  /* stacked cross c_attn: [E][L*2E], [L*2E] */
    /* per layer i, base pointers into the flat buffers; offsets of each tensor within a layer
     * block are given by layer_off[] (elements) in the order of ergm_layer_tensor. */
    const float* layer_f32; const void* layer_b16;
    int64_t layer_stride;     /* elements between layer i and i+1 blocks (negative: reversed order) */
    int64_t layer_off[18];
    /* gradients (f32, same layout as params) */
    float* g_wte; float* g_wpe; float* g_ln_f_w; float* g_ln_f_b; float* g_emo_w;
    float* g_capkv_w; float* g_capkv_b; float* g_layer;
    /* feature projections (feat_dim != n_embd only): visual / audio Conv1D weights [Fd][E] (bf16
     * shadow), biases [E] f32, gradients f32; each bias stored right after its weight */
    const void* vproj_w_b; const float* vproj_b; const void* aproj_w_b; const float* aproj_b;
    float* g_vproj_w; float* g_vproj_b; float* g_aproj_w; float* g_aproj_b;
    /* fp32 master of the stacked caption K/V weight [E][L*2E]; optional, not read by the executor (the
     * fp8 weight quantiser reads the bf16 shadow capkv_w_b) */
    const float* capkv_w;
} ergm_model_params;

typedef enum {
    ERGM_T_LN1_W = 0, ERGM_T_LN1_B, ERGM_T_ATTN_W, ERGM_T_ATTN_B, ERGM_T_APROJ_W, ERGM_T_APROJ_B,
    ERGM_T_LNX_W, ERGM_T_LNX_B, ERGM_T_XQ_W, ERGM_T_XQ_B, ERGM_T_XPROJ_W, ERGM_T_XPROJ_B,
    ERGM_T_LN2_W, ERGM_T_LN2_B, ERGM_T_FC_W, ERGM_T_FC_B, ERGM_T_MPROJ_W, ERGM_T_MPROJ_B,
} ergm_layer_tensor;

/* Bytes of device workspace the executor needs (activations saved for backward + scratch).
 * Shape rules: 2 <= seq <= n_positions, any batch (token counts B*S that are not multiples of 64 run
 * the weight-gradient GEMMs on the register-staged kernel), n_head * 64 == n_embd <= 1024, n_inner and
 * feat_dim multiples of 64; ERGM_EINVAL otherwise. */
size_t ergm_model_workspace_size(const ergm_model_dims* dims);
int ergm_model_create(const ergm_model_dims* dims, const ergm_model_params* params, void* workspace,
                      size_t ws_bytes, ergm_model_plan** out_plan);
int ergm_model_destroy(ergm_model_plan* plan);
/* Inputs for the next forward (device pointers, int64 [B][S]; features f32 or NULL; labels may be
 * NULL for inference).  counts_global: device int[2] the caller filled (ergm_count_valid + optional
 * all-reduce over DP ranks): the LM and the emotion loss means divide by these global counts.     */
/* Optional: a caller-owned byte per padded vocabulary row (n >= vocab_pad).  When set, every training
 * forward writes 1 for the rows its token / token-type / caption lookups touch and 0 elsewhere
 * (stream-ordered, final once the forward returns on its stream).  The lookup gradients of the
 * embedding backward land only in flagged rows of g_wte; all other rows of g_wte are final once
 * the LM-head weight gradient is (after ergm_model_backward_layer(L-2)), which lets an optimizer
 * update them while the rest of the backward runs.  NULL disables. */
int ergm_model_set_row_flags(ergm_model_plan* plan, void* row_flag, int n);
/* Optional (data parallelism): route the lookup gradient sums of the embedding backward to
 * compact[row_pos[row]] (rows of E floats, added onto caller-zeroed rows) instead of adding them to
 * g_wte[row].  row_pos = ergm_rows_scan of the rank-union of the row flags.  NULLs disable. */
int ergm_model_set_lookup_compact(ergm_model_plan* plan, const int* row_pos, float* compact);
/* pos[r] = number of nonzero flags before r (exclusive prefix sum), count[0] = the total. */
int ergm_rows_scan(const void* row_flag, int n, int* pos, int* count, void* stream);
/* For every flagged row r of n: mode 0 zeroes compact[pos[r]]; mode 1 adds it into dst[r]
 * (rows of row_len floats). */
int ergm_rows_compact(const void* row_flag, const int* pos, int n, int row_len, float* compact, float* dst,
                      int mode, void* stream);
int ergm_model_set_inputs(ergm_model_plan* plan, const int64_t* ids, const int64_t* tt,
                          const int64_t* cap_ids, const float* vis, const float* aud,
                          const int64_t* labels, const int64_t* emotion_labels,
                          const int* counts_global);
/* Forward. Outputs (device): logits bf16 [B*S][vocab_pad], emotion logits f32 [B][7],
 * loss parts f32 (ergm_loss_finalize layout: [lm, emotion, total], local contributions over the
 * global normalisers); with `train`, dlogits are prepared for the backward.                      */
int ergm_model_forward(ergm_model_plan* plan, void* logits, float* emo_logits, float* out_loss,
                       int train, void* stream);
/* Backward in stages so a DP caller can overlap communication:
 *   ergm_model_backward_head  — LM head + emotion head + ln_f (grads of wte(part), emo, ln_f)
 *   ergm_model_backward_layer — block `layer` (call for L-1 … 0)
 *   ergm_model_backward_embed — stacked caption K/V projection + embeddings (wte rest, wpe)
 * Weight-gradient GEMMs run on the plan's internal side stream.  Ordering guarantee on `stream`:
 * after backward_layer(l) the gradients of the head stage and of blocks > l are final (block l's
 * own weight gradients are joined by the NEXT stage); after backward_embed every gradient is. */
int ergm_model_backward_head(ergm_model_plan* plan, const float* grad_scale_dev, void* stream);
int ergm_model_backward_layer(ergm_model_plan* plan, int layer, void* stream);
int ergm_model_backward_embed(ergm_model_plan* plan, void* stream);
/* Dropout of the next training forwards (ergm_model_forward with train = 1) and their backward:
 * attn_p = attention probabilities (src/model.py:142), resid_p = the attention / cross-attention /
 * MLP residual branches (:245, :266), embd_p = the embeddings (:506); all 0 = the deterministic path
 * (default).  Masks are ergm_dropout_mask's with this seed and offset (the caller advances offset
 * every training forward), site numbers ERGM_DROP_SITE_*, rows counted from global sample
 * batch_base (data parallelism: rank·batch, so DP ranks draw exactly the masks one process would
 * draw for the concatenated batch).  Inference forwards (train = 0) never drop.                  */
int ergm_model_set_dropout(ergm_model_plan* plan, float attn_p, float resid_p, float embd_p, uint64_t seed,
                           uint32_t offset, int batch_base);
/* Executor-scheduled AdamW (single process).  With a descriptor set, the backward stages also launch the
 * torch.optim.AdamW update (ergm_adamw_step / ergm_adamw_rows arithmetic) of each parameter range as soon as
 * its gradient is final, on an optimizer stream of the plan that waits for the stage's data-gradient work and
 * its weight-gradient mark; ergm_model_backward_embed joins that stream into the caller's, so every update is
 * done, in stream order, when it returns.  Schedule: range k of `ranges` after stage k (0: head + block L-1,
 * …, L-1: block 0, the last after the embedding stage), range L (caption K/V + wpe) after the embedding
 * stage; the tied wte ([vocab_pad][n_embd] at wte_begin): the rows no lookup touched (ergm_model_set_row_flags)
 * after the LM-head weight gradient (stage L-2), the touched rows after the embedding stage (all rows there
 * when no row flags are set).  The descriptor (and its ranges) is copied; set it again every step (lr, step
 * size); NULL disables.  Replaces ergm_amd's per-bucket Python hooks: one Python call per backward stage. */
typedef struct {
    float* param;             /* flat fp32 master */
    const float* grad;        /* flat fp32 gradient */
    float* exp_avg;
    float* exp_avg_sq;
    void* param_bf16;         /* flat bf16 shadow (refreshed by the update), or NULL */
    const int64_t* ranges;    /* [n_ranges][2] element ranges [a, b) */
    int n_ranges;             /* n_layer + 1 */
    int64_t wte_begin;        /* element offset of the tied wte */
    double lr, beta1, beta2, weight_decay;  /* doubles as torch holds them (ABI 5) */
    float eps;
    float step_size;          /* lr / (1 - beta1^t) */
    float bc2_sqrt;           /* sqrt(1 - beta2^t) */
    int max_blocks;           /* grid cap of each update, 0 = none */
    int defer;                /* 1: the updates of blocks 1 … L-1 (and the head) are launched after the embedding
                               * stage instead, in forward order, and NOT joined: the next forward of the plan
                               * waits for each block's update before that block (so they overlap the
                               * latency-bound forward instead of the throughput-bound backward); anything else
                               * that reads the parameters first calls ergm_model_optimizer_join */
} ergm_adamw_desc;
int ergm_model_set_optimizer(ergm_model_plan* plan, const ergm_adamw_desc* opt);
/* Make `stream` wait for every deferred update still pending (no-op when none). */
int ergm_model_optimizer_join(ergm_model_plan* plan, void* stream);
/* Side-stream joins.  per_stage = 1 (default): the ordering guarantee above.  per_stage = 0: the
 * caller's stream does not wait for block l+1's weight gradients at the end of stage l (so the
 * data-gradient chain never idles behind the weight-gradient GEMMs); only backward_embed joins, after
 * which every gradient is final on `stream` as before.  A consumer of block l's gradients (a DP
 * all-reduce, an overlapped optimizer) then makes its stream wait with ergm_model_stage_wait(plan, l,
 * its_stream) after the stage that finalises it was enqueued; stage L+1 = the LM-head (tied wte)
 * weight gradient, L+2 = the caption K/V / projection weight gradients.                             */
int ergm_model_set_side_joins(ergm_model_plan* plan, int per_stage);
/* Trainer metrics on the device (src/main.py:158-169: the running sum of loss.item() and the emotion
 * argmax accuracy): when set, every training forward adds its total loss to loss_acc[0], its LM loss to
 * loss_acc[1] and its number of samples with argmax(emotion_logits) == emotion_labels (first maximum, as
 * torch.argmax) to *correct, in the loss finalisation (no extra launch).  nullptr pointers: off.      */
int ergm_model_set_metrics(ergm_model_plan* plan, float* loss_acc, int64_t* correct);
/* A caller's gradient on the logits of the last training forward (bf16 [B*S][vocab_pad], pad columns 0;
 * src/model.py:698 returns differentiable logits): the next ergm_model_backward_head adds it to the
 * cross-entropy's dlogits (dlogits = bf16(grad_scale · dlogits + grad_logits)) before the LM-head backward
 * GEMMs, then forgets it.  NULL: none (default).  The buffer must stay valid until that call. */
int ergm_model_set_logits_grad(ergm_model_plan* plan, const void* grad_logits);
int ergm_model_stage_wait(ergm_model_plan* plan, int stage, void* stream);

/* Kernel probe for in-loop timing: while set, the executor records `ev_begin` / `ev_end`
 * (hipEvent_t, passed as void*) on the stream immediately around the probed launch:
 *   1 = tied LM-head forward GEMM      2 = LM-head dX GEMM      3 = LM-head dW GEMM
 *   4 = stacked caption-K/V forward GEMM (all blocks)        0 = off                         */
int ergm_model_set_probe(ergm_model_plan* plan, int probe, void* ev_begin, void* ev_end);
/* List probe (bench roofline of a launch class): event pair k is recorded around the k-th launch of the class
 * in the following steps, up to n, and flops[k] (host array, may be NULL) receives its algorithmic FLOPs;
 * ergm_model_probe_count returns how many were recorded.  probe 5 = the weight-gradient GEMMs (every block's
 * Conv1D dW + bias, the stacked caption K/V dW, the LM-head dW), 6 = the block forward Conv1D GEMMs.
 * n = 0 disables. */
int ergm_model_set_probe_list(ergm_model_plan* plan, int probe, void** ev_begin, void** ev_end, double* flops, int n);
int ergm_model_probe_count(const ergm_model_plan* plan);

/* Library information and errors. */
int ergm_version(void);
int ergm_last_error(char* buf, size_t n);

#ifdef __cplusplus
}
#endif
#endif /* ERGM_HIP_H */
