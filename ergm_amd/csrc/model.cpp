// Native executor for the whole fused GPT-2 (ERGM) training step on gfx950.
//
// ergm_model_forward   = GPT2LMHeadModel.forward (src/model.py:654-737): embeddings + fusion
//                        (:459-506), L × GPT2Block (:286-341: self-attn, cross-attn over caption
//                        embeddings, MLP), ln_f (:578), tied LM head (:698), emotion head (:700-701),
//                        LM + emotion CE (:704-713)
// ergm_model_backward_* = loss.backward() (src/main.py:154) in three stages (head, per block, embed)
//                        so a data-parallel caller can all-reduce finished gradient buckets while the
//                        remaining blocks run.
// One C call launches a whole stage (no per-op Python/ctypes overhead); every buffer is caller-owned.
// Design points: the cross-attention K/V projection of the caption embeddings — the same
// tensor in every block (src/model.py:521) — runs as ONE GEMM for all L blocks with the stacked
// weights [E][L·2E]; its backward is split back per block (each block stage issues its slice's dW and
// accumulates its dX into the caption gradient), so none of it waits for the embedding stage.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <new>
#include <vector>

#include "common.h"

using namespace ergm;

namespace ergm {
int layernorm_fwd_ld(const float* x, const float* gamma, const float* beta, void* y, int ldy, float* mean, float* rstd,
                     int rows, int E, float eps, hipStream_t s, void* yq = nullptr, int ldq = 0, float* qscale = nullptr,
                     void* qmx = nullptr, int ld_qmx = 0);
int quant_weights_fp8(const WqJobs& J, hipStream_t s);
int quant_weights_mx(const MxJobs& J, hipStream_t s);
int attn_fwd_mx(const void* q, const void* k, const void* v, void* o, float* lse, int B, int H, int Sq, int Sk, int ldq,
                int ldk, int ldv, int ldo, int causal, const ergm_dropout* dropout, void* keep_bits, uint8_t* qmx,
                uint8_t* qms, int ldqm, int qpitch, hipStream_t s);
bool attn_bwd_fusable(int Sq, int Sk, int K);
int attn_fwd_qgemm(const void* x, int ldx, const void* w, int ldw, const float* bias, int K, void* q, int ldq,
                   const void* k, const void* v, void* o, float* lse, int B, int H, int Sq, int Sk, int ldk, int ldv,
                   int ldo, const ergm_dropout* dropout, void* keep_bits, hipStream_t s);
int attn_bwd_fused(const void* q, const void* k, const void* v, const void* o, const void* dy, int lddy, const void* w,
                   int ldw, int K, const float* lse, void* dq, void* dk, void* dv, int B, int H, int Sq, int Sk, int ldq,
                   int ldk, int ldv, int ldo, int lddq, int lddk, int lddv, int causal, const ergm_dropout* dropout,
                   const void* keep_bits, hipStream_t s);
int quant_rows_mx(const void* X, int x_dtype, int ldx, int rows, int cols, void* Q, int ldq, void* S, int lds,
                  hipStream_t s);
int quant_rows_fp8(const void* X, int x_dtype, int ldx, int rows, int cols, void* Q, int ldq, float* scale,
                   hipStream_t s);
int fill_ones_col(void* p, int rows, int ld, int col, hipStream_t s);
int ln_bwd_nparts(int rows);
int ln_bwd_rows_per_part();
int layernorm_bwd_main(const void* dy, int dy_bf16, const float* x, const float* mean, const float* rstd,
                       const float* gamma, float* dres, void* dres_bf16, float* part_g, float* part_b, int rows, int E,
                       hipStream_t s, const DropSite& drop, int drop_res, void* qmx, void* qmx_s, int ld_qs);
int layernorm_param_reduce(const float* part_g, const float* part_b, int rows, int E, float* dgamma, float* dbeta,
                           hipStream_t s);
int layernorm_param_reduce_n(int n, const float* const* part_g, const float* const* part_b, int rows, int E,
                             float* const* dgamma, float* const* dbeta, hipStream_t s);
int loss_finalize_metrics(const float* row_loss, int T, const int* n_valid_global, const float* emo_loss_sum,
                          const int* n_valid_emo, float* out, float* loss_acc, int64_t* correct,
                          const float* emo_logits, const int64_t* emo_labels, int B, int C, hipStream_t s);
int gemm_dw_pair(const ergm_gemm_desc* const d[2], const void* const A[2], const void* const B[2], void* const C[2],
                 void* stream, bool launch);
int dlogits_add(void* dl, const void* g, const float* scale, size_t n, hipStream_t s);
int embed_fwd_ld(const int64_t* ids, const int64_t* tt, const int64_t* cap_ids, const float* wte, const float* wpe,
                 const float* vis, int ld_vis, const float* aud, float* h0, void* cap, int ld_cap, int B, int S, int E,
                 int V, hipStream_t s, const DropSite& drop);
int embed_bwd_sort(const int64_t* ids, const int64_t* tt, const int64_t* cap_ids, int T, int V, uint64_t* keys,
                   uint8_t* row_flag, int n_flag, hipStream_t s);
int embed_sort_capacity(int T);
int embed_bwd_sums(const uint64_t* keys, int B, int S, int E, const float* dh0, const float* dcap, float* dwte,
                   float* dwpe, float* part, const int* row_pos, hipStream_t s);
int feat_pack(const float* vis, int ld_vis, const float* aud, void* out, int B, int Bp, int Fd, int ld, hipStream_t s);
int proj_grad_pack(const float* dh0, void* d, int B, int Bp, int S, int E, hipStream_t s);
}  // namespace ergm

struct LayerActs {
    __bf16 *ln1, *lnx, *ln2;
    float *m1, *r1, *mx, *rx, *m2, *r2;
    __bf16 *qkv, *ao, *xq, *xo, *pre, *act;  // pre: gelu_new' of the c_fc pre-activation (GELU backward factor)
    float *lse, *xlse;
};

// fp8 (config 5) copies of one block's six Conv1D weights, transposed to [N][K] e4m3 with per-column
// scales (order: c_attn, attn c_proj, q_attn, cross c_proj, c_fc, mlp c_proj), and their amax scratch
struct LayerW8 {
    uint8_t* w[6];
    float* sc[6];
    uint8_t* sx[6];  // MX-fp8: e8m0 scale per (column, 32-row block), [N][K/32]
    unsigned* amax;
    int amax_n;
};

// one pending weight-gradient GEMM (dw_gemm / dw_flush)
struct DwJob {
    int M, N;
    const __bf16* A;
    int lda;
    const __bf16* dY;
    int ldy;
    float* gW;
    float* gB;
    int ldc;  // row stride of gW (N, or the stacked matrix's width for a column slice)
};

struct ergm_model_plan {
    ergm_model_dims d;
    ergm_model_params p;
    int T, L2E;
    // Activations that feed a weight-gradient GEMM carry a constant ones column (index E or F) so the
    // dW GEMM over K+1 rows also yields the bias gradient (each bias is stored right after its weight).
    int XE, XF;
    bool fused_bias;  // the ones-column layout holds (every bias right after its weight): dW over M+1 rows
    bool ones_pending;  // the ones columns are written by the first forward, on the caller's stream
    // activations
    float** resid;  // 3L+1 residual-stream tensors [T][E] f32
    std::vector<float*> resid_v;
    std::vector<LayerActs> la;
    __bf16 *cap, *kv_all, *lnf;
    float *mf, *rf;
    __bf16* dlogits;
    float *row_loss, *emo_sum, *emo_tmp;
    int* n_valid_local;
    // feature projections (feat_dim != n_embd): bf16 operands [2][Bp][Fd+8] (visual rows, then audio
    // rows; ones column at Fd for the fused bias gradient; batch padded to Bp = round64(B) zero rows so
    // the weight-gradient GEMM's contraction over the batch is a whole K tile), projected vectors f32
    // [2][Bp][E] (what the embedding kernel injects), their bf16 gradients [2][Bp][E]
    bool proj;
    int Fd, Bp;
    __bf16* feat_b16;
    float* proj_out;
    __bf16* dproj;
    // fp8 forward (dims.fp8): per-block weight copies re-quantised at every forward on the side stream
    // (ev_wq[l] marks block l's), the caption K/V weights likewise, and the transient row-quantised
    // activations (main stream: one buffer reused block after block; side stream: the captions)
    bool f8;
    // MX-fp8 (default; ERGM_FP8_MX=0: the per-row / per-column scales): e8m0 scales per 32-element K block of
    // every activation row and weight column, consumed by the MFMA (ergm_gemm_mx); the LayerNorms and the c_fc
    // GELU epilogue write their MX copies themselves, the weights are quantised in one pass (no amax pass)
    bool mx = true;
    std::vector<LayerW8> w8;
    uint8_t *capkv8, *qa, *qf, *qcap;
    float *capkv8_s, *sa, *sf, *scap;
    uint8_t *capkv8_x, *xa, *xf, *xcap;
    unsigned* capkv_amax;
    std::vector<hipEvent_t> ev_wq;
    // the caption K/V projection of block l done on the side stream (kv_per_block): block l's cross-attention waits
    // for ev_kv[l] only, so the later blocks' projections overlap the latency-bound forward
    std::vector<hipEvent_t> ev_kv;
    bool kv_per_block;  // one caption K/V GEMM per block (ERGM_KV_PER_BLOCK=0: one GEMM for all blocks)
    // per_stage_join: the caller's stream waits for block l+1's side-stream weight gradients at the end
    // of stage l (ergm_model_backward_layer's ordering guarantee); 0 = only the embedding stage joins,
    // consumers of a block's gradients wait with ergm_model_stage_wait instead
    bool per_stage_join;
    // forward batch-half chains: the second runs on fwd2 (ev_f2: fork, embedding done, chain done);
    // the backward's data-gradient chains likewise (bwd_forked: the second chain is running, forked
    // after the head stage and joined by the embedding stage)
    int fwd_chains, bwd_chains;
    bool attn_fuse;  // attention backward with the c_proj data-gradient GEMM inside (attn_bwd_fused, S <= 128)
    bool xq_fuse;    // cross-attention forward with the query projection inside (attn_fwd_qgemm; bf16 forward)
    bool dw_group;  // weight-gradient pairs issued behind one side-stream fork run as ONE grouped launch when both
                    // qualify (gemm_dw_pair)
    // stages between a block's backward and its AdamW launch (opt_after_layer): 2 measured best (vs 1: C2 -0.4 %,
    // C5 -0.6 %; 0 slower, profiles/r02_experiments.txt)
    int opt_lag = 2;
    std::vector<DwJob> dw_pend;
    bool bwd_forked;
    hipStream_t fwd2;
    hipEvent_t ev_f2[3];
    char* scratch3;
    // lookups sorted by vocabulary row (computed during the training forward, used by the embedding
    // backward) and the caller's optional touched-row flags (one byte per padded vocab row)
    uint64_t* keys;
    uint8_t* row_flag;
    // optional compact destination of the lookup gradient sums (data parallelism, ergm_hip.h)
    const int* row_pos;
    float* lookup_compact;
    // backward scratch
    float *dh, *dy, *dcap, *delta;
    __bf16* dyb;  // the block LayerNorms' incoming gradient: their data-gradient GEMM's bf16 output (ln_f's: dy, f32)
    bool ln_dy_f32;  // ERGM_LN_DY_F32=1: the block LayerNorms read an f32 data-gradient GEMM output (dy) instead
    bool bind_forks;  // fork points bound to the producing launch (arm_fork); ERGM_BIND_FORKS=0: recorded events only
    bool lm_dw_first;  // the LM-head dW is forked before the LM-head dX GEMM, so the two run together (+0.5 % per step
                       // at C2 over six interleaved pairs, profiles/r06_ab{2,3}.txt); ERGM_LMHEAD_DW_FIRST=0: after it
    __bf16 *d_o, *dkv_all;
    // dY operands of the weight-gradient GEMMs get one buffer per use (no reuse), so the dW GEMMs can
    // run on the side stream while the data-gradient chain continues: dhb[i] = bf16 grad of resid[i].
    std::vector<__bf16*> dhb, dpre, dxq, dqkv;
    // dγ/dβ partials of each LayerNorm backward (one slot per LN, reduced on the side stream)
    std::vector<float*> ln_part;
    int ln_slot;
    int ln_pending;  // LayerNorm backwards whose dγ/dβ reduction is not yet launched (ln_reduce_flush)
    const float* lnr_pg[4];
    const float* lnr_pb[4];
    float* lnr_dg[4];
    float* lnr_db[4];
    char *scratch, *scratch2;
    size_t scratch_bytes;
    // Two HIP streams: the caller's stream runs the critical chain; `side` runs weight-gradient GEMMs
    // (and the stacked caption K/V GEMM in forward), forked/joined with events.
    hipStream_t side;
    hipEvent_t ev_fork;  // fork points are bound to the producing launch (common.h ERGM_LAUNCH) or recorded
    // the stage's final fork point from the caller's stream (ln_reduce_flush), valid until the native call that took
    // it returns: the optimizer updates launched behind the stage wait on it (opt_wait) instead of a new marker
    hipEvent_t stage_pt = nullptr;
    std::vector<hipEvent_t> ev_join;  // one per backward stage (L layers + head + embed)
    // inputs
    const int64_t *ids, *tt, *cap_ids, *labels, *emo_labels;
    const float *vis, *aud;
    const int* n_valid;  // [0] valid LM labels, [1] valid emotion labels (global under DP)
    const void* logits_grad = nullptr;  // ergm_model_set_logits_grad: caller's bf16 gradient on the logits (next backward)
    float* metric_loss = nullptr;       // ergm_model_set_metrics: [0] += loss, [1] += LM loss per training forward
    int64_t* metric_correct = nullptr;  // += emotion argmax hits per training forward
    bool have_fwd;
    // dropout (src/model.py:142,245,266,506): probabilities, seed and forward number set by the caller
    // (ergm_model_set_dropout) for the next training forward; `drop_on` is latched by that forward and
    // read by its backward.  abits: the attention forwards' keep bits, [2L][B·H·S][mwords] u64.
    float p_attn, p_resid, p_embd;
    uint64_t drop_seed;
    uint32_t drop_offset;
    int b_base;  // global batch index of local sample 0 (data-parallel rank offset)
    bool drop_on;
    uint64_t* abits;
    int mwords;
    // kernel probe (bench timing): one event pair (probes 1-4) or a list (probe 5: every weight-gradient
    // GEMM launch, with its algorithmic FLOPs)
    int probe;
    hipEvent_t ev_begin, ev_end;
    hipEvent_t* evl_b;
    hipEvent_t* evl_e;
    double* evl_flops;
    int evl_n, evl_k;
    // launch class of the GEMMs being enqueued (LaunchClass; 1 = block forward GEMMs, list probe 6)
    int launch_cls;
    // executor-scheduled AdamW (ergm_model_set_optimizer): descriptor copy, its ranges, the optimizer stream
    // and the main-stream marks it waits for (one per update of a step)
    bool opt_on;
    ergm_adamw_desc opt;
    std::vector<int64_t> opt_ranges;
    hipStream_t opt_s;
    std::vector<hipEvent_t> ev_opt;
    int opt_k;
    std::vector<hipEvent_t> ev_upd;  // deferred update of block l done (opt.defer)
    std::vector<char> upd_pending;   // block l's deferred update not yet waited for by a forward
    // dry-run sizing
    bool dry;
    size_t need;
};

namespace {

struct Carver {
    char* base;
    size_t off = 0;
    template <typename T>
    T* take(size_t n) {
        off = (off + 255) & ~(size_t)255;
        T* p = base ? reinterpret_cast<T*>(base + off) : nullptr;
        off += n * sizeof(T);
        return p;
    }
};

// Lay out every activation buffer; returns bytes used (scratch excluded).
size_t carve(ergm_model_plan* P, char* base) {
    const ergm_model_dims& d = P->d;
    const size_t T = (size_t)d.batch * d.seq, E = d.n_embd, F = d.n_inner, L = d.n_layer;
    const size_t BHS = (size_t)d.batch * d.n_head * d.seq;
    const size_t XE = E + 8, XF = F + 8;
    P->XE = (int)XE;
    P->XF = (int)XF;
    Carver c{base};
    P->resid_v.assign(3 * L + 1, nullptr);
    for (size_t i = 0; i < 3 * L + 1; ++i) P->resid_v[i] = c.take<float>(T * E);
    P->la.assign(L, LayerActs{});
    for (size_t l = 0; l < L; ++l) {
        LayerActs& a = P->la[l];
        a.ln1 = c.take<__bf16>(T * XE); a.lnx = c.take<__bf16>(T * XE); a.ln2 = c.take<__bf16>(T * XE);
        a.m1 = c.take<float>(T); a.r1 = c.take<float>(T); a.mx = c.take<float>(T);
        a.rx = c.take<float>(T); a.m2 = c.take<float>(T); a.r2 = c.take<float>(T);
        a.qkv = c.take<__bf16>(T * 3 * E); a.ao = c.take<__bf16>(T * XE);
        a.xq = c.take<__bf16>(T * E); a.xo = c.take<__bf16>(T * XE);
        a.pre = c.take<__bf16>(T * F); a.act = c.take<__bf16>(T * XF);
        a.lse = c.take<float>(BHS); a.xlse = c.take<float>(BHS);
    }
    P->cap = c.take<__bf16>(T * XE);
    P->kv_all = c.take<__bf16>(T * 2 * E * L);
    P->lnf = c.take<__bf16>(T * E);
    P->mf = c.take<float>(T); P->rf = c.take<float>(T);
    P->dlogits = c.take<__bf16>(T * d.vocab_pad);
    P->row_loss = c.take<float>(T);
    P->emo_sum = c.take<float>(4);
    P->emo_tmp = c.take<float>((size_t)d.batch * 16 + 8);
    P->n_valid_local = c.take<int>(4);
    P->f8 = d.fp8 != 0;
    P->w8.assign(P->f8 ? L : 0, LayerW8{});
    P->capkv8 = P->qa = P->qf = P->qcap = nullptr;
    P->capkv8_s = P->sa = P->sf = P->scap = nullptr;
    P->capkv8_x = P->xa = P->xf = P->xcap = nullptr;
    P->capkv_amax = nullptr;
    if (P->f8) {
        const size_t KN[6][2] = {{E, 3 * E}, {E, E}, {E, E}, {E, E}, {E, F}, {F, E}};
        for (size_t l = 0; l < L; ++l) {
            LayerW8& w = P->w8[l];
            int na = 0;
            for (int i = 0; i < 6; ++i) {
                w.w[i] = c.take<uint8_t>(KN[i][0] * KN[i][1]);
                w.sc[i] = c.take<float>(KN[i][1]);
                w.sx[i] = c.take<uint8_t>(KN[i][0] / 32 * KN[i][1]);
                na += (int)KN[i][1];
            }
            w.amax = c.take<unsigned>(na);
            w.amax_n = na;
        }
        P->capkv8 = c.take<uint8_t>((size_t)2 * E * L * E);
        P->capkv8_s = c.take<float>((size_t)2 * E * L);
        P->capkv_amax = c.take<unsigned>((size_t)2 * E * L);
        P->qa = c.take<uint8_t>(T * E);
        P->sa = c.take<float>(T);
        P->qf = c.take<uint8_t>(T * F);
        P->sf = c.take<float>(T);
        P->qcap = c.take<uint8_t>(T * E);
        P->scap = c.take<float>(T);
        P->capkv8_x = c.take<uint8_t>((size_t)2 * E * L * (E / 32));
        P->xa = c.take<uint8_t>(T * (E / 32));
        P->xf = c.take<uint8_t>(T * (F / 32));
        P->xcap = c.take<uint8_t>(T * (E / 32));
    }
    P->Fd = d.feat_dim > 0 ? d.feat_dim : (int)E;
    P->proj = d.has_features && P->Fd != (int)E;
    P->Bp = (d.batch + 63) / 64 * 64;
    if (P->proj) {
        P->feat_b16 = c.take<__bf16>((size_t)2 * P->Bp * (P->Fd + 8));
        P->proj_out = c.take<float>((size_t)2 * P->Bp * E);
        P->dproj = c.take<__bf16>((size_t)2 * P->Bp * E);
    } else {
        P->feat_b16 = nullptr;
        P->proj_out = nullptr;
        P->dproj = nullptr;
    }
    P->keys = c.take<uint64_t>(embed_sort_capacity(T));
    P->mwords = (d.seq + 63) / 64;
    P->abits = c.take<uint64_t>((size_t)2 * L * BHS * P->mwords);
    P->dh = c.take<float>(T * E); P->dy = c.take<float>(T * E); P->dyb = c.take<__bf16>(T * E); P->dcap = c.take<float>(T * E);
    P->delta = c.take<float>(BHS);
    P->d_o = c.take<__bf16>(T * E);
    P->dkv_all = c.take<__bf16>(T * 2 * E * L);
    P->dhb.assign(3 * L + 1, nullptr);
    for (size_t i = 0; i < 3 * L + 1; ++i) P->dhb[i] = c.take<__bf16>(T * E);
    P->ln_part.assign(3 * L + 1, nullptr);
    for (size_t i = 0; i < 3 * L + 1; ++i) P->ln_part[i] = c.take<float>((size_t)2 * ln_bwd_nparts((int)T) * E);
    P->dpre.assign(L, nullptr); P->dxq.assign(L, nullptr); P->dqkv.assign(L, nullptr);
    for (size_t l = 0; l < L; ++l) {
        P->dpre[l] = c.take<__bf16>(T * F);
        P->dxq[l] = c.take<__bf16>(T * E);
        P->dqkv[l] = c.take<__bf16>(T * 3 * E);
    }
    P->scratch = c.take<char>(0);
    P->resid = P->resid_v.data();
    return c.off;
}

inline int ws_need(ergm_model_plan* P, size_t bytes) {
    if (P->dry) {
        P->need = std::max(P->need, bytes);
        return ERGM_OK;
    }
    ERGM_CHECK_ARG(bytes <= P->scratch_bytes, "model: scratch %zu < %zu", P->scratch_bytes, bytes);
    return ERGM_OK;
}

// Dropout descriptor of `site` for rows starting at global row `row0` (p == 0: off).  The residual
// sites count token rows ((b_base + b)·S + s), the attention sites (b·H + h)·S + q rows.
ergm_dropout drop_desc(const ergm_model_plan* P, uint32_t site, float p, int64_t row0) {
    ergm_dropout d{};
    d.seed = P->drop_seed;
    d.offset = P->drop_offset;
    d.site = site;
    d.p = P->drop_on ? p : 0.f;
    d.row0 = row0;
    return d;
}
ergm_dropout resid_drop(const ergm_model_plan* P, int resid_index, int b0) {
    return drop_desc(P, (uint32_t)resid_index, resid_index == 0 ? P->p_embd : P->p_resid,
                     (int64_t)(P->b_base + b0) * P->d.seq);
}
ergm_dropout attn_drop(const ergm_model_plan* P, int l, int cross, int b0) {
    return drop_desc(P, ERGM_DROP_SITE_ATTN(P->d.n_layer, l, cross), P->p_attn,
                     (int64_t)(P->b_base + b0) * P->d.n_head * P->d.seq);
}
uint64_t* attn_bits(const ergm_model_plan* P, int l, int cross, int b0) {
    if (P->dry) return nullptr;
    const size_t per = (size_t)P->d.batch * P->d.n_head * P->d.seq * P->mwords;
    return P->abits + (2 * (size_t)l + cross) * per + (size_t)b0 * P->d.n_head * P->d.seq * P->mwords;
}

// Records the probe events around one launch: the single pair when `id` is the active probe (1-4), or the
// next pair of the list when `id` is the active list probe (5: weight-gradient GEMMs, 6: block forward GEMMs).
struct Probe {
    hipEvent_t end = nullptr;
    hipStream_t s;
    Probe(ergm_model_plan* P, int id, hipStream_t s_, double flops = 0.0) : s(s_) {
        if (P->dry || P->probe != id) return;
        if (P->evl_n == 0) {
            if (!P->ev_begin) return;
            (void)hipEventRecord(P->ev_begin, s);
            end = P->ev_end;
        } else if (P->evl_k < P->evl_n) {
            const int k = P->evl_k++;
            (void)hipEventRecord(P->evl_b[k], s);
            end = P->evl_e[k];
            if (P->evl_flops) P->evl_flops[k] = flops;
        }
    }
    ~Probe() {
        if (end) (void)hipEventRecord(end, s);
    }
};

int gemm(ergm_model_plan* P, hipStream_t s, int M, int N, int K, const void* A, int lda, int al, const void* B,
         int ldb, int bl, void* C, int ldc, int cdt, int epi, const float* bias = nullptr, const void* aux = nullptr,
         int ld_aux = 0, void* aux_out = nullptr, int ld_aux_out = 0, const float* alpha_dev = nullptr,
         const ergm_dropout* dropout = nullptr, float* bias_grad = nullptr) {
    ergm_gemm_desc g;
    memset(&g, 0, sizeof(g));
    g.M = M; g.N = N; g.K = K; g.lda = lda; g.ldb = ldb; g.ldc = ldc;
    g.a_layout = al; g.b_layout = bl; g.c_dtype = cdt; g.epilogue = epi; g.alpha = 1.0f;
    g.bias = bias; g.aux = aux; g.ld_aux = ld_aux; g.aux_out = aux_out; g.ld_aux_out = ld_aux_out;
    g.split_k = 0; g.alpha_dev = alpha_dev; g.dropout = dropout; g.bias_grad = bias_grad;
    size_t w = ergm_gemm_workspace_size(&g);
    ERGM_TRY(ws_need(P, w));
    if (P->dry) return ERGM_OK;
    Probe pr(P, P->launch_cls == 1 ? 6 : -1, s, 2.0 * M * N * K);
    char* ws = (s != nullptr && s == P->side) ? P->scratch2 : (s != nullptr && s == P->fwd2) ? P->scratch3 : P->scratch;
    return ergm_gemm(&g, A, B, C, ws, P->scratch_bytes, s);
}

// fp8 forward GEMM: C[M][N] = epi(sa[m]·sb[n]·A8[m][:]·B8t[n][:]) (both operands k-contiguous, K bytes)
// MX (P->mx): the scales are the e8m0 block scales ax [M][K/32] / bx [N][K/32]; qo / qox (BIAS_GELU only): the MX
// copy of the bf16 output [M][N] / [M][N/32] for the next fp8 GEMM.
int gemm8(ergm_model_plan* P, hipStream_t s, int M, int N, int K, const uint8_t* A, const float* sa, const uint8_t* ax,
          const uint8_t* Bt, const float* sb, const uint8_t* bx, void* C, int ldc, int cdt, int epi, const float* bias,
          const void* aux = nullptr, int ld_aux = 0, void* aux_out = nullptr, int ld_aux_out = 0,
          const ergm_dropout* dropout = nullptr, uint8_t* qo = nullptr, uint8_t* qox = nullptr, int b_pitch = 0) {
    if (P->dry) return ERGM_OK;
    ergm_gemm_desc g;
    memset(&g, 0, sizeof(g));
    g.M = M; g.N = N; g.K = K; g.lda = K; g.ldb = K; g.ldc = ldc;
    g.a_layout = ERGM_MK; g.b_layout = ERGM_NK; g.c_dtype = cdt; g.epilogue = epi; g.alpha = 1.0f;
    g.bias = bias; g.aux = aux; g.ld_aux = ld_aux; g.aux_out = aux_out; g.ld_aux_out = ld_aux_out;
    g.dropout = dropout;
    // MX scale pitches (mx_sidx): activation rows (A, the MX copy of C) are token rows of a T-row buffer, B is a
    // weight copy with exactly N rows (b_pitch: rows of a larger copy B is a row slice of)
    if (P->mx) return ergm_gemm_mx(&g, A, ax, P->T, Bt, bx, b_pitch ? b_pitch : N, C, qo, qox, N, P->T, s);
    return ergm_gemm_f8(&g, A, sa, Bt, sb, C, s);
}
// Row quantisation of an fp8 GEMM's activation operand (attention outputs, caption embeddings; the GELU output
// too without MX): per-row scale `sf` or MX block scales `sx`.
int quant_act(ergm_model_plan* P, const void* X, int ldx, int rows, int cols, uint8_t* q, float* sf, uint8_t* sx,
              hipStream_t s) {
    if (P->mx) return quant_rows_mx(X, ERGM_BF16, ldx, rows, cols, q, cols, sx, P->T, s);
    return quant_rows_fp8(X, ERGM_BF16, ldx, rows, cols, q, cols, sf, s);
}


// Executor streams: non-blocking (they order themselves with the caller's stream through events).
hipError_t make_stream(hipStream_t* s) { return hipStreamCreateWithFlags(s, hipStreamNonBlocking); }

// Fork/join events order two streams of the same device: device-scope release is enough, and skipping
// the system-scope fence avoids an L2 writeback at every record on the critical stream.
constexpr unsigned kSyncEv = hipEventDisableTiming | hipEventDisableSystemFence;

// An event that completes with everything enqueued so far on `s`: the fork point armed before the stage's last
// launch on s when that launch carried it and nothing else was enqueued on s since (arm_fork: no marker packet on
// s), else `ev` recorded on s.  The caller waits on it at once: ev_fork is re-bound by the next arm.
hipEvent_t stream_point(ergm_model_plan* P, hipStream_t s, hipEvent_t ev) {
    (void)P;
    hipEvent_t e = bind_take(s);
    if (!e && hipEventRecord(ev, s) == hipSuccess) e = ev;
    return e;
}
// Bind the next fork point of `s` to the launches that follow on s (the stage's producer of the fork).
void arm_fork(ergm_model_plan* P, hipStream_t s) {
    if (!P->dry && P->bind_forks) bind_arm(s, P->ev_fork);
}

// Make the side stream wait for everything issued so far on `s` (the producer of a dW GEMM's dY).
int fork_side(ergm_model_plan* P, hipStream_t s) {
    if (P->dry) return ERGM_OK;
    hipEvent_t e = stream_point(P, s, P->ev_fork);
    if (!e || hipStreamWaitEvent(P->side, e, 0) != hipSuccess) return fail(ERGM_EHIP, "model: stream fork failed");
    return ERGM_OK;
}

// The backward's data-gradient chains: every kernel of a block's data-gradient path is row- (or
// batch-) separable, so like the forward it runs as two concurrent chains over the two halves of the
// batch (the caller's stream and P->fwd2) and writes disjoint rows of the same buffers; the weight-
// gradient GEMMs (side stream, contraction over all tokens) wait for both.  One chain when the batch
// does not split into halves whose token counts are multiples of the LayerNorm-backward partial block.
struct Chains {
    int n;
    hipStream_t s[2];
    int b0[2], nb[2];
};
Chains bwd_chains(const ergm_model_plan* P, hipStream_t s) {
    Chains c{};
    const int B = P->d.batch, S = P->d.seq;
    const bool two = !P->dry && P->bwd_chains >= 2 && B >= 2 && ((B / 2) * S) % 8 == 0;
    c.n = two ? 2 : 1;
    c.s[0] = s;
    c.s[1] = two ? P->fwd2 : s;
    c.b0[0] = 0;
    c.nb[0] = two ? B / 2 : B;
    c.b0[1] = c.nb[0];
    c.nb[1] = B - c.nb[0];
    return c;
}
int fork_side(ergm_model_plan* P, const Chains& c) {
    for (int i = 0; i < c.n; ++i) ERGM_TRY(fork_side(P, c.s[i]));
    return ERGM_OK;
}

// Record stage event `k` on the side stream / make `s` wait for a recorded stage event.
int side_mark(ergm_model_plan* P, int k) {
    if (P->dry) return ERGM_OK;
    return hipEventRecord(P->ev_join[k], P->side) == hipSuccess ? ERGM_OK : fail(ERGM_EHIP, "model: event record");
}
int join_side(ergm_model_plan* P, hipStream_t s, int k) {
    if (P->dry) return ERGM_OK;
    return hipStreamWaitEvent(s, P->ev_join[k], 0) == hipSuccess ? ERGM_OK : fail(ERGM_EHIP, "model: stream join");
}

// Tags the GEMMs enqueued in its scope with a launch class (list probe 6 times the block forward GEMMs, class 1).
struct LaunchClass {
    ergm_model_plan* P;
    int prev;
    LaunchClass(ergm_model_plan* P_, int c) : P(P_), prev(P_->launch_cls) { P->launch_cls = c; }
    ~LaunchClass() { P->launch_cls = prev; }
};

// Weight gradient of a Conv1D: gW[M][N] = Aᵀ·dY over the T tokens (A = the layer input, [T][lda]) and its
// bias gradient gB[N] = Σ_t dY[t][n].  With fused_bias the A operand's column M is all ones and gB == gW + M·N,
// so one GEMM over M+1 rows writes [gW; gB] (the extra tile row runs beside the others); otherwise the GEMM
// sums gB from the dY fragments it stages (ergm_gemm_desc.bias_grad: measured equal at C2 but +4 % step time
// at C4, where its last tile row carrying the column sums through 64 K steps becomes the long pole).
double dw_flops(const ergm_model_plan* P, const DwJob& j) { return 2.0 * j.M * j.N * P->T + (double)j.N * P->T; }
void dw_desc(const ergm_model_plan* P, const DwJob& j, ergm_gemm_desc& g) {
    memset(&g, 0, sizeof(g));
    g.M = P->fused_bias ? j.M + 1 : j.M;
    g.N = j.N; g.K = P->T; g.lda = j.lda; g.ldb = j.ldy; g.ldc = j.ldc;
    g.a_layout = ERGM_KM; g.b_layout = ERGM_KN; g.c_dtype = ERGM_F32; g.epilogue = ERGM_EPI_NONE;
    g.alpha = 1.0f;
    g.bias_grad = P->fused_bias ? nullptr : j.gB;
}
int dw_launch(ergm_model_plan* P, hipStream_t s, const DwJob& j) {
    Probe pr(P, 5, s, dw_flops(P, j));
    ergm_gemm_desc g;
    dw_desc(P, j, g);
    const size_t w = ergm_gemm_workspace_size(&g);
    ERGM_TRY(ws_need(P, w));
    if (P->dry) return ERGM_OK;
    return ergm_gemm(&g, j.A, j.dY, j.gW, s == P->side ? P->scratch2 : P->scratch, P->scratch_bytes, s);
}
// Two pending weight-gradient GEMMs as ONE grouped launch (gemm_dw_pair) when they plan to the same unsplit
// configuration: each alone has fewer tiles than the chip has CUs (ERGM_DW_GROUP=0: two launches).
// Returns ERGM_EUNSUPPORTED when the pair does not qualify (nothing launched).
int dw_launch_pair(ergm_model_plan* P, hipStream_t s, const DwJob& j0, const DwJob& j1) {
    if (!P->dw_group) return ERGM_EUNSUPPORTED;
    ergm_gemm_desc g[2];
    dw_desc(P, j0, g[0]);
    dw_desc(P, j1, g[1]);
    const ergm_gemm_desc* d[2] = {&g[0], &g[1]};
    const void* A[2] = {j0.A, j1.A};
    const void* B[2] = {j0.dY, j1.dY};
    void* C[2] = {j0.gW, j1.gW};
    ERGM_TRY(gemm_dw_pair(d, A, B, C, s, false));
    Probe pr(P, 5, s, dw_flops(P, j0) + dw_flops(P, j1));
    return gemm_dw_pair(d, A, B, C, s, true);
}
// Queue a weight-gradient GEMM; dw_flush launches the queue on the side stream behind ONE fork from the data-
// gradient chain(s).
int dw_gemm(ergm_model_plan* P, const Chains& ch, int M, int N, const __bf16* A, int lda, const __bf16* dY, int ldy,
            float* gW, float* gB, int ldc = 0) {
    const DwJob j{M, N, A, lda, dY, ldy, gW, gB, ldc ? ldc : N};
    if (P->dry) return dw_launch(P, ch.s[0], j);
    P->dw_pend.push_back(j);
    return ERGM_OK;
}
// Launch the pending weight-gradient GEMMs on the side stream behind ONE fork from the data-gradient
// chain(s) (every dY they read is complete there): one event record + wait instead of one per GEMM.
int dw_flush(ergm_model_plan* P, const Chains& ch) {
    if (P->dw_pend.empty()) return ERGM_OK;
    ERGM_TRY(fork_side(P, ch));
    size_t i = 0;
    for (; i + 1 < P->dw_pend.size(); i += 2) {
        const int r = dw_launch_pair(P, P->side, P->dw_pend[i], P->dw_pend[i + 1]);
        if (r == ERGM_EUNSUPPORTED) break;
        ERGM_TRY(r);
    }
    for (; i < P->dw_pend.size(); ++i) ERGM_TRY(dw_launch(P, P->side, P->dw_pend[i]));
    P->dw_pend.clear();
    return ERGM_OK;
}

// LayerNorm backward on the critical chain(s): rows [r0, r0 + rows) of the residual stream; its dγ/dβ
// partials (one per 8-row block, so every chain writes its own partial rows and the reduce sees the
// one-chain partials bit for bit) go to a per-LN slot (nothing later overwrites them) and are reduced
// on the side stream by ln_reduce_flush, which batches the pending LayerNorms of a block into one launch.
int ln_bwd_rows(ergm_model_plan* P, hipStream_t s, const float* x, const float* mean, const float* rstd,
                const float* gamma, __bf16* dh_b, int slot, int r0, int rows) {
    if (P->dry) return ERGM_OK;
    const int T = P->T, E = P->d.n_embd;
    float* pg = P->ln_part[slot];
    float* pb = pg + (size_t)ln_bwd_nparts(T) * E;
    const size_t o = (size_t)r0 * E, po = (size_t)(r0 / ln_bwd_rows_per_part()) * E;
    // dh_b feeds the residual branch that produced this residual-stream tensor (slot = its index):
    // through that branch's dropout.  Slot 0 (the embeddings) has no bf16 consumer: there the final dh
    // itself goes through the embedding dropout (src/model.py:506), folded into this pass.
    const ergm_dropout dd = resid_drop(P, slot, r0 / P->d.seq);
    const int fin = slot == 0;
    // the block LayerNorms read their data-gradient GEMM's output rounded to bf16 — a rounding the fp32 reference
    // does not have (src/main.py trains without autocast), kept because it halves the LayerNorm backward's dy traffic
    // (-0.3 % C2 step, profiles/r05_experiments.txt #11) at no measurable cost in the parity margins (DESIGN.md §10;
    // ERGM_LN_DY_F32=1 keeps dy in f32); ln_f (slot 3L) reads the f32 sum of the LM-head and emotion-head gradients
    const bool yb = slot != 3 * P->d.n_layer && !P->ln_dy_f32;
    return layernorm_bwd_main(yb ? (const void*)(P->dyb + o) : (const void*)(P->dy + o), yb, x + o, mean + r0, rstd + r0, gamma, P->dh + o, fin ? nullptr : dh_b + o,
                              pg + po, pb + po, rows, E, s, drop_site_of(&dd, E), fin, nullptr, nullptr, T);
}
int ln_reduce_add(ergm_model_plan* P, int slot, float* dgamma, float* dbeta) {
    if (P->dry) return ERGM_OK;
    ERGM_CHECK_ARG(P->ln_pending < 4, "model: too many pending LayerNorm reductions");
    float* pg = P->ln_part[slot];
    const int k = P->ln_pending++;
    P->lnr_pg[k] = pg; P->lnr_pb[k] = pg + (size_t)ln_bwd_nparts(P->T) * P->d.n_embd;
    P->lnr_dg[k] = dgamma; P->lnr_db[k] = dbeta;
    return ERGM_OK;
}
int ln_bwd(ergm_model_plan* P, hipStream_t s, const float* x, const float* mean, const float* rstd, const float* gamma,
           float* dgamma, float* dbeta, __bf16* dh_b, int slot) {
    ERGM_TRY(ln_bwd_rows(P, s, x, mean, rstd, gamma, dh_b, slot, 0, P->T));
    return ln_reduce_add(P, slot, dgamma, dbeta);
}

int ln_reduce_flush(ergm_model_plan* P, const Chains& ch) {
    if (P->dry || P->ln_pending == 0) return ERGM_OK;
    {  // behind the chains' LayerNorm backwards (their partials)
        hipEvent_t e = stream_point(P, ch.s[0], P->ev_fork);
        if (!e || hipStreamWaitEvent(P->side, e, 0) != hipSuccess) return fail(ERGM_EHIP, "model: stream fork failed");
        for (int i = 1; i < ch.n; ++i) ERGM_TRY(fork_side(P, ch.s[i]));
        // the end of the stage on ch.s[0] (nothing more is enqueued there in this call) — unless a second chain's fork
        // re-recorded ev_fork on fwd2 just now: then opt_wait records its own point on the caller's stream
        P->stage_pt = ch.n == 1 ? e : nullptr;
    }
    const int n = P->ln_pending;
    P->ln_pending = 0;
    return layernorm_param_reduce_n(n, P->lnr_pg, P->lnr_pb, P->T, P->d.n_embd, P->lnr_dg, P->lnr_db, P->side);
}


inline const float* LF(const ergm_model_plan* P, int l, int t) {
    return P->p.layer_f32 + (int64_t)l * P->p.layer_stride + P->p.layer_off[t];
}
inline const __bf16* LB(const ergm_model_plan* P, int l, int t) {
    return reinterpret_cast<const __bf16*>(P->p.layer_b16) + (int64_t)l * P->p.layer_stride + P->p.layer_off[t];
}
inline float* LG(const ergm_model_plan* P, int l, int t) {
    return P->p.g_layer + (int64_t)l * P->p.layer_stride + P->p.layer_off[t];
}

// Re-quantise block l's six Conv1D weights (bf16 shadow → transposed e4m3 + column scales: half the bytes
// of the f32 master, and the values the bf16 backward GEMMs use) on `ss` and
// mark ev_wq[l]; the block's forward waits for that mark.
int quant_layer_weights(ergm_model_plan* P, int l, hipStream_t ss) {
    if (P->dry) return ERGM_OK;
    const int E = P->d.n_embd, F = P->d.n_inner;
    LayerW8& w = P->w8[l];
    const int tens[6] = {ERGM_T_ATTN_W, ERGM_T_APROJ_W, ERGM_T_XQ_W, ERGM_T_XPROJ_W, ERGM_T_FC_W, ERGM_T_MPROJ_W};
    const int K[6] = {E, E, E, E, E, F}, N[6] = {3 * E, E, E, E, F, E};
    if (P->mx) {  // one pass: block scales from each 32-row block's own maxima
        MxJobs J{};
        J.n = 6;
        for (int i = 0; i < 6; ++i) {
            J.j[i] = MxJob{LB(P, l, tens[i]), w.w[i], w.sx[i], N[i], K[i], N[i], K[i], N[i], 0};
        }
        ERGM_TRY(quant_weights_mx(J, ss));
        return hipEventRecord(P->ev_wq[l], ss) == hipSuccess ? ERGM_OK : fail(ERGM_EHIP, "model: event record");
    }
    if (hipMemsetAsync(w.amax, 0, (size_t)w.amax_n * 4, ss) != hipSuccess) return fail(ERGM_EHIP, "model: memset");
    WqJobs J{};
    J.n = 6;
    unsigned* am = w.amax;
    for (int i = 0; i < 6; ++i) {
        J.j[i] = WqJob{LB(P, l, tens[i]), w.w[i], w.sc[i], am, N[i], K[i], N[i], K[i], 0, 0, 1};
        am += N[i];
    }
    ERGM_TRY(quant_weights_fp8(J, ss));
    return hipEventRecord(P->ev_wq[l], ss) == hipSuccess ? ERGM_OK : fail(ERGM_EHIP, "model: event record");
}

int do_forward(ergm_model_plan* P, void* logits, float* emo_logits, float* out_loss, int train, hipStream_t s);
int wait_update(ergm_model_plan* P, int l, hipStream_t s);
int do_backward_head(ergm_model_plan* P, const float* gscale, hipStream_t s);
int do_backward_layer(ergm_model_plan* P, int l, hipStream_t s);
int do_backward_embed(ergm_model_plan* P, hipStream_t s);

}  // namespace

extern "C" size_t ergm_model_workspace_size(const ergm_model_dims* dims) {
    if (!dims) return 0;
    ergm_model_plan P{};
    P.d = *dims;
    memset(&P.p, 0, sizeof(P.p));
    P.T = dims->batch * dims->seq;
    P.L2E = 2 * dims->n_embd * dims->n_layer;
    size_t act = carve(&P, nullptr);
    P.dry = true;
    P.fused_bias = false;  // size for the in-GEMM bias path (its split-K partials)
    P.need = ergm_embed_bwd_workspace_size(P.T);
    P.labels = P.emo_labels = nullptr;
    P.fwd2 = nullptr;
    for (int chains = 1; chains <= 2; ++chains) {  // size for the whole batch and for its halves
        P.fwd_chains = chains;
        do_forward(&P, nullptr, nullptr, nullptr, 1, nullptr);
    }
    do_backward_head(&P, nullptr, nullptr);
    do_backward_layer(&P, 0, nullptr);
    do_backward_embed(&P, nullptr);
    return ((act + 255) & ~(size_t)255) + 3 * (((P.need + 255) & ~(size_t)255) + 256);
}

extern "C" int ergm_model_create(const ergm_model_dims* dims, const ergm_model_params* params, void* ws,
                                 size_t ws_bytes, ergm_model_plan** out) {
    ERGM_CHECK_ARG(dims && params && ws && out, "model_create: null argument");
    const ergm_model_dims& d = *dims;
    ERGM_CHECK_ARG(d.n_embd > 0 && d.n_head > 0 && d.n_embd == 64 * d.n_head,
                   "model_create: head_dim must be 64 (n_embd=%d n_head=%d)", d.n_embd, d.n_head);
    ERGM_CHECK_ARG(d.n_embd % 64 == 0 && d.n_embd <= 1024, "model_create: n_embd=%d unsupported", d.n_embd);
    ERGM_CHECK_ARG(d.n_inner % 64 == 0, "model_create: n_inner must be a multiple of 64");
    ERGM_CHECK_ARG(d.vocab > 0 && d.vocab_pad >= d.vocab && d.vocab_pad % 64 == 0, "model_create: bad vocab_pad");
    ERGM_CHECK_ARG(d.batch > 0 && d.seq >= 2 && d.seq <= d.n_positions, "model_create: bad batch/seq");
    ERGM_CHECK_ARG(d.n_layer > 0, "model_create: n_layer must be > 0");
    ERGM_CHECK_ARG(d.feat_dim >= 0 && d.feat_dim % 64 == 0, "model_create: feat_dim must be a multiple of 64");
    ERGM_CHECK_ARG(!d.fp8 || (d.n_embd % 128 == 0 && d.n_inner % 128 == 0),
                   "model_create: fp8 needs n_embd, n_inner multiples of 128");
    if (d.has_features && d.feat_dim > 0 && d.feat_dim != d.n_embd) {
        const ergm_model_params& q = *params;
        ERGM_CHECK_ARG(q.vproj_w_b && q.vproj_b && q.aproj_w_b && q.aproj_b && q.g_vproj_w && q.g_aproj_w,
                       "model_create: feat_dim %d != n_embd needs the projection parameters", d.feat_dim);
        const int64_t wsz = (int64_t)d.feat_dim * d.n_embd;
        ERGM_CHECK_ARG(q.g_vproj_b == q.g_vproj_w + wsz && q.g_aproj_b == q.g_aproj_w + wsz,
                       "model_create: projection bias gradients must follow their weights");
    }
    size_t need = ergm_model_workspace_size(dims);
    ERGM_CHECK_ARG(ws_bytes >= need, "model_create: workspace %zu < %zu bytes", ws_bytes, need);
    auto* P = new (std::nothrow) ergm_model_plan();
    if (!P) return fail(ERGM_EINVAL, "model_create: out of host memory");
    P->d = d;
    P->p = *params;
    P->T = d.batch * d.seq;
    P->L2E = 2 * d.n_embd * d.n_layer;
    size_t act = carve(P, reinterpret_cast<char*>(ws));
    act = (act + 255) & ~(size_t)255;
    P->scratch_bytes = (ws_bytes - act) / 3 & ~(size_t)255;
    P->scratch = reinterpret_cast<char*>(ws) + act;
    P->scratch2 = P->scratch + P->scratch_bytes;
    P->scratch3 = P->scratch2 + P->scratch_bytes;
    P->side = nullptr;
    P->ev_fork = nullptr;
    P->ev_join.assign(d.n_layer + 3, nullptr);
    bool ok = make_stream(&P->side) == hipSuccess &&
              hipEventCreateWithFlags(&P->ev_fork, kSyncEv) == hipSuccess;
    for (auto& e : P->ev_join) ok = ok && hipEventCreateWithFlags(&e, kSyncEv) == hipSuccess;
    // two forward chains over the batch halves (one chain measured +3-5 %, three level, four +20 %: round 2)
    P->fwd_chains = 2;
    if (const char* e = getenv("ERGM_FWD_CHAINS")) P->fwd_chains = std::max(1, std::min(2, atoi(e)));
    // two backward chains measured slower at C2 (6.27 vs 5.85 ms/step: the GPU is already throughput-
    // saturated and the host enqueue grows, profiles/r02_bwd_chains_ab.txt): ERGM_BWD_CHAINS=2 enables
    P->bwd_chains = 1;
    if (const char* e = getenv("ERGM_BWD_CHAINS")) P->bwd_chains = atoi(e);
    if (const char* e = getenv("ERGM_FP8_MX")) P->mx = atoi(e) != 0;
    P->ln_dy_f32 = false;
    if (const char* e = getenv("ERGM_LN_DY_F32")) P->ln_dy_f32 = atoi(e) != 0;
    P->bind_forks = true;
    if (const char* e = getenv("ERGM_BIND_FORKS")) P->bind_forks = atoi(e) != 0;
    P->lm_dw_first = true;
    if (const char* e = getenv("ERGM_LMHEAD_DW_FIRST")) P->lm_dw_first = atoi(e) != 0;
    // grouped pairs measured -0.2 % (C2) / -0.5 % (C4) per step at E = 768 but +0.9 % at C5 (E = 1024, whose
    // qualifying pairs are the 1025 x {1024, 3072} shapes on 128x128 tiles): on below E = 1024
    P->dw_group = d.n_embd < 1024;
    if (const char* e = getenv("ERGM_DW_GROUP")) P->dw_group = atoi(e) != 0;
    // the c_proj dX GEMM inside the short attention backward: bitwise the two-launch form (ERGM_ATTN_FUSE=0
    // restores it for the A/B and the parity test)
    P->attn_fuse = attn_bwd_fusable(d.seq, d.seq, d.n_embd);
    if (const char* e = getenv("ERGM_ATTN_FUSE")) P->attn_fuse = P->attn_fuse && atoi(e) != 0;
    // the query projection inside the cross-attention forward (bf16 forward only; ERGM_XQ_FUSE=0: two launches)
    P->xq_fuse = !P->f8 && d.n_embd % 64 == 0;
    if (const char* e = getenv("ERGM_XQ_FUSE")) P->xq_fuse = P->xq_fuse && atoi(e) != 0;
    P->bwd_forked = false;
    P->per_stage_join = true;
    P->fwd2 = nullptr;
    for (auto& e : P->ev_f2) e = nullptr;
    ok = ok && make_stream(&P->fwd2) == hipSuccess;
    for (auto& e : P->ev_f2) ok = ok && hipEventCreateWithFlags(&e, kSyncEv) == hipSuccess;
    P->ev_wq.assign(P->f8 ? d.n_layer : 0, nullptr);
    for (auto& e : P->ev_wq) ok = ok && hipEventCreateWithFlags(&e, kSyncEv) == hipSuccess;
    P->kv_per_block = true;
    if (const char* e = getenv("ERGM_KV_PER_BLOCK")) P->kv_per_block = atoi(e) != 0;
    if (const char* e = getenv("ERGM_OPT_LAG")) P->opt_lag = std::max(0, std::min(4, atoi(e)));  // A/B only
    P->ev_kv.assign(P->kv_per_block ? d.n_layer : 0, nullptr);
    for (auto& e : P->ev_kv) ok = ok && hipEventCreateWithFlags(&e, kSyncEv) == hipSuccess;
    if (!ok) {
        ergm_model_destroy(P);
        return fail(ERGM_EHIP, "model_create: stream/event creation failed");
    }
    P->dry = false;
    P->need = 0;
    P->have_fwd = false;
    P->ln_pending = 0;
    // Fused bias gradients need every Conv1D bias stored right after its weight (ergm_amd/params.py lays the
    // flat buffers out that way) and a ones column in the activations (producers write columns < E / < F
    // only); other layouts take the in-GEMM column sums (ergm_gemm_desc.bias_grad).  The first forward
    // writes the ones columns on its own stream: the caller's allocator may hand over a workspace whose
    // previous owner still has work queued on that stream, which a write from here (legacy null stream,
    // unordered with non-blocking streams) would race — and lose the columns to (profiles/r05_experiments.txt #29).
    P->ones_pending = true;
    {
        const int64_t E = d.n_embd, F = d.n_inner;
        const int64_t* o = P->p.layer_off;
        auto follows = [&](int w, int b, int64_t K, int64_t N) { return o[b] == o[w] + K * N; };
        P->fused_bias = follows(ERGM_T_ATTN_W, ERGM_T_ATTN_B, E, 3 * E) && follows(ERGM_T_APROJ_W, ERGM_T_APROJ_B, E, E) &&
                        follows(ERGM_T_XQ_W, ERGM_T_XQ_B, E, E) && follows(ERGM_T_XPROJ_W, ERGM_T_XPROJ_B, E, E) &&
                        follows(ERGM_T_FC_W, ERGM_T_FC_B, E, F) && follows(ERGM_T_MPROJ_W, ERGM_T_MPROJ_B, F, E) &&
                        P->p.g_capkv_b == P->p.g_capkv_w + E * P->L2E;
    }
    P->ids = P->tt = P->cap_ids = P->labels = P->emo_labels = nullptr;
    P->vis = P->aud = nullptr;
    P->row_flag = nullptr;
    P->row_pos = nullptr;
    P->lookup_compact = nullptr;
    P->n_valid = nullptr;
    P->probe = 0;
    P->launch_cls = 0;
    P->opt_on = false;
    P->opt_s = nullptr;
    P->opt_k = 0;
    P->ev_begin = P->ev_end = nullptr;
    P->evl_b = P->evl_e = nullptr;
    P->evl_flops = nullptr;
    P->evl_n = P->evl_k = 0;
    P->p_attn = P->p_resid = P->p_embd = 0.f;
    P->drop_seed = 0;
    P->drop_offset = 0;
    P->b_base = 0;
    P->drop_on = false;
    *out = P;
    return ERGM_OK;
}

extern "C" int ergm_model_destroy(ergm_model_plan* P) {
    if (!P) return ERGM_OK;
    if (P->side) hipStreamSynchronize(P->side);
    for (auto e : P->ev_join)
        if (e) hipEventDestroy(e);
    for (auto e : P->ev_wq)
        if (e) hipEventDestroy(e);
    for (auto e : P->ev_kv)
        if (e) hipEventDestroy(e);
    for (auto e : P->ev_f2)
        if (e) hipEventDestroy(e);
    if (P->fwd2) {
        hipStreamSynchronize(P->fwd2);
        hipStreamDestroy(P->fwd2);
    }
    if (P->opt_s) {
        hipStreamSynchronize(P->opt_s);
        hipStreamDestroy(P->opt_s);
    }
    for (auto e : P->ev_opt)
        if (e) hipEventDestroy(e);
    for (auto e : P->ev_upd)
        if (e) hipEventDestroy(e);
    if (P->ev_fork) hipEventDestroy(P->ev_fork);
    if (P->side) hipStreamDestroy(P->side);
    delete P;
    return ERGM_OK;
}

extern "C" int ergm_model_set_probe(ergm_model_plan* P, int probe, void* ev_begin, void* ev_end) {
    ERGM_CHECK_ARG(P && probe >= 0 && probe <= 4, "model_set_probe: bad probe");
    ERGM_CHECK_ARG(probe == 0 || (ev_begin && ev_end), "model_set_probe: events required");
    P->probe = probe;
    P->ev_begin = reinterpret_cast<hipEvent_t>(ev_begin);
    P->ev_end = reinterpret_cast<hipEvent_t>(ev_end);
    P->evl_n = P->evl_k = 0;
    return ERGM_OK;
}

extern "C" int ergm_model_set_probe_list(ergm_model_plan* P, int probe, void** ev_begin, void** ev_end, double* flops,
                                         int n) {
    ERGM_CHECK_ARG(P && n >= 0 && (n == 0 || (ev_begin && ev_end)) && (probe == 5 || probe == 6),
                   "model_set_probe_list: bad argument");
    P->probe = n > 0 ? probe : 0;
    P->ev_begin = P->ev_end = nullptr;
    P->evl_b = reinterpret_cast<hipEvent_t*>(ev_begin);
    P->evl_e = reinterpret_cast<hipEvent_t*>(ev_end);
    P->evl_flops = flops;
    P->evl_n = n;
    P->evl_k = 0;
    return ERGM_OK;
}

extern "C" int ergm_model_probe_count(const ergm_model_plan* P) { return P ? P->evl_k : 0; }

extern "C" int ergm_model_set_dropout(ergm_model_plan* P, float attn_p, float resid_p, float embd_p, uint64_t seed,
                                      uint32_t offset, int batch_base) {
    ERGM_CHECK_ARG(P, "model_set_dropout: null plan");
    ERGM_CHECK_ARG(attn_p >= 0.f && attn_p < 1.f && resid_p >= 0.f && resid_p < 1.f && embd_p >= 0.f && embd_p < 1.f,
                   "model_set_dropout: probabilities must be in [0, 1)");
    ERGM_CHECK_ARG(batch_base >= 0, "model_set_dropout: batch_base must be >= 0");
    ERGM_CHECK_ARG(attn_p == 0.f || P->d.seq <= 1024, "model_set_dropout: attention dropout needs seq <= 1024");
    P->p_attn = attn_p;
    P->p_resid = resid_p;
    P->p_embd = embd_p;
    P->drop_seed = seed;
    P->drop_offset = offset;
    P->b_base = batch_base;
    return ERGM_OK;
}

extern "C" int ergm_model_set_logits_grad(ergm_model_plan* P, const void* grad_logits) {
    ERGM_CHECK_ARG(P, "model_set_logits_grad: null plan");
    ERGM_CHECK_ARG(!grad_logits || aligned16(grad_logits), "model_set_logits_grad: 16-byte alignment");
    P->logits_grad = grad_logits;
    return ERGM_OK;
}

extern "C" int ergm_model_set_metrics(ergm_model_plan* P, float* loss_acc, int64_t* correct) {
    ERGM_CHECK_ARG(P, "model_set_metrics: null plan");
    P->metric_loss = loss_acc;
    P->metric_correct = correct;
    return ERGM_OK;
}

extern "C" int ergm_model_set_side_joins(ergm_model_plan* P, int per_stage) {
    ERGM_CHECK_ARG(P, "model_set_side_joins: null plan");
    P->per_stage_join = per_stage != 0;
    return ERGM_OK;
}

extern "C" int ergm_model_stage_wait(ergm_model_plan* P, int stage, void* stream) {
    ERGM_CHECK_ARG(P && stage >= 0 && stage < P->d.n_layer + 3 && stage != P->d.n_layer,
                   "model_stage_wait: stage in [0, L) or L+1, L+2");
    return hipStreamWaitEvent(as_stream(stream), P->ev_join[stage], 0) == hipSuccess
               ? ERGM_OK
               : fail(ERGM_EHIP, "model_stage_wait: hipStreamWaitEvent");
}

extern "C" int ergm_model_set_row_flags(ergm_model_plan* P, void* row_flag, int n) {
    ERGM_CHECK_ARG(P, "model_set_row_flags: null plan");
    ERGM_CHECK_ARG(!row_flag || n >= P->d.vocab_pad, "model_set_row_flags: need %d bytes (got %d)", P->d.vocab_pad, n);
    P->row_flag = reinterpret_cast<uint8_t*>(row_flag);
    return ERGM_OK;
}

extern "C" int ergm_model_set_lookup_compact(ergm_model_plan* P, const int* row_pos, float* compact) {
    ERGM_CHECK_ARG(P, "model_set_lookup_compact: null plan");
    ERGM_CHECK_ARG((row_pos == nullptr) == (compact == nullptr), "model_set_lookup_compact: both or neither");
    P->row_pos = row_pos;
    P->lookup_compact = compact;
    return ERGM_OK;
}

extern "C" int ergm_model_set_inputs(ergm_model_plan* P, const int64_t* ids, const int64_t* tt,
                                     const int64_t* cap_ids, const float* vis, const float* aud,
                                     const int64_t* labels, const int64_t* emotion_labels, const int* counts_global) {
    ERGM_CHECK_ARG(P && ids && cap_ids, "model_set_inputs: input_ids and caption_ids are required");
    ERGM_CHECK_ARG((vis == nullptr) == (aud == nullptr), "model_set_inputs: visual/audio features go together");
    ERGM_CHECK_ARG(!vis || P->d.has_features, "model_set_inputs: plan built without features");
    ERGM_CHECK_ARG(!(labels || emotion_labels) || counts_global, "model_set_inputs: labels need counts_global");
    P->ids = ids; P->tt = tt; P->cap_ids = cap_ids; P->vis = vis; P->aud = aud;
    P->labels = labels; P->emo_labels = emotion_labels; P->n_valid = counts_global;
    return ERGM_OK;
}

namespace {
// One block's forward (src/model.py:286-341) over the batch rows [b0, b0+nb) on stream s: every
// kernel is row- (or batch-) separable, so two such chains over disjoint halves of the batch run
// concurrently on two streams and write disjoint rows of the same activation buffers — the backward
// sees the full-batch layout unchanged.
// `part` selects one launch group (0-10, in chain order: LN1, c_attn, attention, attn c_proj, LN_x, q,
// cross-attention, cross c_proj, LN2, c_fc, mlp c_proj) so that the caller can interleave the chains
// launch by launch; -1 issues the whole block.
int fwd_block(ergm_model_plan* P, int l, hipStream_t s, int b0, int nb, int part = -1) {
    LaunchClass lc(P, 1);
    auto on = [part](int k) { return part < 0 || part == k; };
    if (on(0)) ERGM_TRY(wait_update(P, l, s));  // a deferred optimizer update of this block's parameters
    const ergm_model_dims& d = P->d;
    const int E = d.n_embd, F = d.n_inner, L = d.n_layer, H = d.n_head, S = d.seq, L2E = P->L2E;
    const int T = nb * S;
    const size_t r0 = (size_t)b0 * S, XE = P->XE, XF = P->XF;
    const LayerActs& a0 = P->la[l];
    LayerActs a = a0;
    if (!P->dry) {
        a.ln1 += r0 * XE; a.lnx += r0 * XE; a.ln2 += r0 * XE;
        a.m1 += r0; a.r1 += r0; a.mx += r0; a.rx += r0; a.m2 += r0; a.r2 += r0;
        a.qkv += r0 * 3 * E; a.ao += r0 * XE; a.xq += r0 * E; a.xo += r0 * XE;
        a.pre += r0 * F; a.act += r0 * XF;
        a.lse += (size_t)b0 * H * S; a.xlse += (size_t)b0 * H * S;
    }
    float* x0 = P->dry ? nullptr : P->resid[3 * l] + r0 * E;
    float* x1 = P->dry ? nullptr : P->resid[3 * l + 1] + r0 * E;
    float* x2 = P->dry ? nullptr : P->resid[3 * l + 2] + r0 * E;
    float* x3 = P->dry ? nullptr : P->resid[3 * l + 3] + r0 * E;
    // fp8 (config 5): every Conv1D below consumes row-quantised activations (the LayerNorms write
    // their fp8 copy themselves, attention / GELU outputs go through quant_rows_fp8) and block l's
    // re-quantised weights, which the side stream marks ready with ev_wq[l]
    const bool f8 = P->f8;
    const LayerW8* w8 = f8 && !P->dry ? &P->w8[l] : nullptr;
    uint8_t* qa = f8 && !P->dry ? P->qa + r0 * E : nullptr;
    uint8_t* qf = f8 && !P->dry ? P->qf + r0 * F : nullptr;
    float* sa = f8 && !P->dry ? P->sa + r0 : nullptr;
    float* sf = f8 && !P->dry ? P->sf + r0 : nullptr;
    uint8_t* xa = f8 && !P->dry ? P->xa + r0 * 4 : nullptr;  // MX block scales of qa / qf rows (pitch T, mx_sidx)
    uint8_t* xf = f8 && !P->dry ? P->xf + r0 * 4 : nullptr;
    float* lsa = P->mx ? nullptr : sa;  // the LayerNorms' fp8 copy: per-row scale or MX block scales
    uint8_t* lxa = P->mx ? xa : nullptr;
    if (on(0) && w8 && hipStreamWaitEvent(s, P->ev_wq[l], 0) != hipSuccess) return fail(ERGM_EHIP, "model: stream wait");
    // dropout sites of this block over the chain's rows (src/model.py:142 probabilities, :245 / :266
    // residual branches)
    const ergm_dropout dr_attn = resid_drop(P, 3 * l + 1, b0), dr_cross = resid_drop(P, 3 * l + 2, b0),
                       dr_mlp = resid_drop(P, 3 * l + 3, b0);
    const ergm_dropout dp_self = attn_drop(P, l, 0, b0), dp_cross = attn_drop(P, l, 1, b0);
    // self-attention sub-block (src/model.py:297-309)
    if (on(0) && !P->dry)
        ERGM_TRY(layernorm_fwd_ld(x0, LF(P, l, ERGM_T_LN1_W), LF(P, l, ERGM_T_LN1_B), a.ln1, P->XE, a.m1, a.r1, T, E,
                                  d.eps, s, qa, E, lsa, lxa, P->T));
    if (on(1)) {
        if (f8)
            ERGM_TRY(gemm8(P, s, T, 3 * E, E, qa, sa, xa, w8 ? w8->w[0] : nullptr, w8 ? w8->sc[0] : nullptr,
                           w8 ? w8->sx[0] : nullptr, a.qkv, 3 * E, ERGM_BF16, ERGM_EPI_BIAS, LF(P, l, ERGM_T_ATTN_B)));
        else
            ERGM_TRY(gemm(P, s, T, 3 * E, E, a.ln1, P->XE, ERGM_MK, LB(P, l, ERGM_T_ATTN_W), 3 * E, ERGM_KN, a.qkv, 3 * E,
                          ERGM_BF16, ERGM_EPI_BIAS, LF(P, l, ERGM_T_ATTN_B)));
    }
    // MX: the attention kernels write the c_proj GEMMs' MX operand themselves
    const bool amx = f8 && P->mx;
    if (on(2) && !P->dry)
        ERGM_TRY(attn_fwd_mx(a.qkv, a.qkv + E, a.qkv + 2 * E, a.ao, a.lse, nb, H, S, S, 3 * E, 3 * E, 3 * E, P->XE, 1,
                             &dp_self, attn_bits(P, l, 0, b0), amx ? qa : nullptr, amx ? xa : nullptr, E, P->T, s));
    if (on(3)) {
        if (f8) {
            if (!P->dry && !amx) ERGM_TRY(quant_act(P, a.ao, P->XE, T, E, qa, sa, xa, s));
            ERGM_TRY(gemm8(P, s, T, E, E, qa, sa, xa, w8 ? w8->w[1] : nullptr, w8 ? w8->sc[1] : nullptr,
                           w8 ? w8->sx[1] : nullptr, x1, E, ERGM_F32, ERGM_EPI_BIAS_RESID, LF(P, l, ERGM_T_APROJ_B), x0, E,
                           nullptr, 0, &dr_attn));
        } else {
            ERGM_TRY(gemm(P, s, T, E, E, a.ao, P->XE, ERGM_MK, LB(P, l, ERGM_T_APROJ_W), E, ERGM_KN, x1, E, ERGM_F32,
                          ERGM_EPI_BIAS_RESID, LF(P, l, ERGM_T_APROJ_B), x0, E, nullptr, 0, nullptr, &dr_attn));
        }
    }
    // cross-attention over caption embeddings (src/model.py:311-329)
    if (on(4) && !P->dry)
        ERGM_TRY(layernorm_fwd_ld(x1, LF(P, l, ERGM_T_LNX_W), LF(P, l, ERGM_T_LNX_B), a.lnx, P->XE, a.mx, a.rx, T, E,
                                  d.eps, s, qa, E, lsa, lxa, P->T));
    if (on(5) && !P->xq_fuse) {
        if (f8)
            ERGM_TRY(gemm8(P, s, T, E, E, qa, sa, xa, w8 ? w8->w[2] : nullptr, w8 ? w8->sc[2] : nullptr,
                           w8 ? w8->sx[2] : nullptr, a.xq, E, ERGM_BF16, ERGM_EPI_BIAS, LF(P, l, ERGM_T_XQ_B)));
        else
            ERGM_TRY(gemm(P, s, T, E, E, a.lnx, P->XE, ERGM_MK, LB(P, l, ERGM_T_XQ_W), E, ERGM_KN, a.xq, E, ERGM_BF16,
                          ERGM_EPI_BIAS, LF(P, l, ERGM_T_XQ_B)));
    }
    const __bf16* kl = P->dry ? nullptr : P->kv_all + r0 * L2E + (size_t)l * 2 * E;
    if (on(6) && !P->dry) {  // the caption K/V of this block (kv_per_block) or of every block (side stream)
        if (P->kv_per_block) {
            if (hipStreamWaitEvent(s, P->ev_kv[l], 0) != hipSuccess) return fail(ERGM_EHIP, "model: stream wait");
        } else if (l == 0) {
            ERGM_TRY(join_side(P, s, L));
        }
    }
    if (on(6) && !P->dry) {
        if (P->xq_fuse)  // q = LN_x·Wq + bq formed inside the cross-attention forward
            ERGM_TRY(attn_fwd_qgemm(a.lnx, P->XE, LB(P, l, ERGM_T_XQ_W), E, LF(P, l, ERGM_T_XQ_B), E, a.xq, E, kl,
                                    kl + E, a.xo, a.xlse, nb, H, S, S, L2E, L2E, P->XE, &dp_cross,
                                    attn_bits(P, l, 1, b0), s));
        else
            ERGM_TRY(attn_fwd_mx(a.xq, kl, kl + E, a.xo, a.xlse, nb, H, S, S, E, L2E, L2E, P->XE, 0, &dp_cross,
                                 attn_bits(P, l, 1, b0), amx ? qa : nullptr, amx ? xa : nullptr, E, P->T, s));
    }
    if (on(7)) {
        if (f8) {
            if (!P->dry && !amx) ERGM_TRY(quant_act(P, a.xo, P->XE, T, E, qa, sa, xa, s));
            ERGM_TRY(gemm8(P, s, T, E, E, qa, sa, xa, w8 ? w8->w[3] : nullptr, w8 ? w8->sc[3] : nullptr,
                           w8 ? w8->sx[3] : nullptr, x2, E, ERGM_F32, ERGM_EPI_BIAS_RESID, LF(P, l, ERGM_T_XPROJ_B), x1, E,
                           nullptr, 0, &dr_cross));
        } else {
            ERGM_TRY(gemm(P, s, T, E, E, a.xo, P->XE, ERGM_MK, LB(P, l, ERGM_T_XPROJ_W), E, ERGM_KN, x2, E, ERGM_F32,
                          ERGM_EPI_BIAS_RESID, LF(P, l, ERGM_T_XPROJ_B), x1, E, nullptr, 0, nullptr, &dr_cross));
        }
    }
    // MLP (src/model.py:331-334, 262-267)
    if (on(8) && !P->dry)
        ERGM_TRY(layernorm_fwd_ld(x2, LF(P, l, ERGM_T_LN2_W), LF(P, l, ERGM_T_LN2_B), a.ln2, P->XE, a.m2, a.r2, T, E,
                                  d.eps, s, qa, E, lsa, lxa, P->T));
    if (f8) {
        if (on(9)) {
            // MX: the GELU epilogue writes the MX copy of its output itself (no quantisation pass)
            ERGM_TRY(gemm8(P, s, T, F, E, qa, sa, xa, w8 ? w8->w[4] : nullptr, w8 ? w8->sc[4] : nullptr,
                           w8 ? w8->sx[4] : nullptr, a.act, P->XF, ERGM_BF16, ERGM_EPI_BIAS_GELU, LF(P, l, ERGM_T_FC_B),
                           nullptr, 0, a.pre, F, nullptr, P->mx ? qf : nullptr, P->mx ? xf : nullptr));
            if (!P->dry && !P->mx) ERGM_TRY(quant_rows_fp8(a.act, ERGM_BF16, P->XF, T, F, qf, F, sf, s));
        }
        if (on(10))
            ERGM_TRY(gemm8(P, s, T, E, F, qf, sf, xf, w8 ? w8->w[5] : nullptr, w8 ? w8->sc[5] : nullptr,
                           w8 ? w8->sx[5] : nullptr, x3, E, ERGM_F32, ERGM_EPI_BIAS_RESID, LF(P, l, ERGM_T_MPROJ_B), x2, E,
                           nullptr, 0, &dr_mlp));
    } else {
        if (on(9))
            ERGM_TRY(gemm(P, s, T, F, E, a.ln2, P->XE, ERGM_MK, LB(P, l, ERGM_T_FC_W), F, ERGM_KN, a.act, P->XF,
                          ERGM_BF16, ERGM_EPI_BIAS_GELU, LF(P, l, ERGM_T_FC_B), nullptr, 0, a.pre, F));
        if (on(10))
            ERGM_TRY(gemm(P, s, T, E, F, a.act, P->XF, ERGM_MK, LB(P, l, ERGM_T_MPROJ_W), E, ERGM_KN, x3, E, ERGM_F32,
                          ERGM_EPI_BIAS_RESID, LF(P, l, ERGM_T_MPROJ_B), x2, E, nullptr, 0, nullptr, &dr_mlp));
    }
    (void)L;
    return ERGM_OK;
}

// LM-head column split: the vocabulary-wide GEMM runs 256x256 tiles, one per CU per round; the leading
// n0 columns are the largest multiple of 256 whose tile count fills whole rounds of 256 CUs, the
// remaining columns (the partial last round) run as a second, small-tile GEMM spread over all CUs.
int lmhead_split_cols(int T, int Vp) {
    const int rows = (T + 255) / 256;
    int q = 256;  // column tiles per whole number of rounds: 256 / gcd(rows, 256)
    for (int r = rows; r % 2 == 0 && q > 1; r /= 2) q /= 2;
    const int n0 = (Vp / 256 / q) * q * 256;
    return (n0 > 0 && Vp - n0 >= 256) ? n0 : Vp;
}

int do_forward(ergm_model_plan* P, void* logits, float* emo_logits, float* out_loss, int train, hipStream_t s) {
    const ergm_model_dims& d = P->d;
    P->drop_on = train != 0 && (P->p_attn > 0.f || P->p_resid > 0.f || P->p_embd > 0.f);
    const int T = P->T, E = d.n_embd, L = d.n_layer, B = d.batch, S = d.seq;
    const int L2E = P->L2E;
    const ergm_model_params& p = P->p;

    const float* vis_in = P->vis;
    const float* aud_in = P->aud;
    int ld_vis = d.ld_vis;
    if (P->proj && (P->dry || P->vis)) {
        // build-side feature projections (config 5): [Bp][Fd]·[Fd][E] + b per modality, MFMA GEMMs
        const int Fd = P->Fd, Bp = P->Bp, ldf = P->Fd + 8;
        if (!P->dry) ERGM_TRY(feat_pack(P->vis, d.ld_vis, P->aud, P->feat_b16, B, Bp, Fd, ldf, s));
        ERGM_TRY(gemm(P, s, Bp, E, Fd, P->feat_b16, ldf, ERGM_MK, p.vproj_w_b, E, ERGM_KN, P->proj_out, E, ERGM_F32,
                      ERGM_EPI_BIAS, p.vproj_b));
        ERGM_TRY(gemm(P, s, Bp, E, Fd, P->feat_b16 ? P->feat_b16 + (size_t)Bp * ldf : nullptr, ldf, ERGM_MK,
                      p.aproj_w_b, E, ERGM_KN, P->proj_out ? P->proj_out + (size_t)Bp * E : nullptr, E, ERGM_F32,
                      ERGM_EPI_BIAS, p.aproj_b));
        vis_in = P->proj_out;
        aud_in = P->proj_out ? P->proj_out + (size_t)Bp * E : nullptr;
        ld_vis = E;
    }
    // Two concurrent chains over the two halves of the batch (main stream: rows of batch [0, B0);
    // P->fwd2: [B0, B)): the forward is a serial chain of mostly latency-bound kernels, and a second
    // independent chain fills the CUs the first leaves idle.  nchain = 1 when B = 1 (or disabled).
    const int nchain = std::max(1, std::min(P->fwd_chains, B));
    int bsplit[3];
    for (int c = 0; c <= nchain; ++c) bsplit[c] = c * B / nchain;
    hipStream_t cs[2] = {s, P->dry ? s : P->fwd2};
    hipEvent_t ev_emb[2] = {nullptr, P->ev_f2[1]};
    hipEvent_t ev_done[2] = {nullptr, P->ev_f2[2]};
    auto embed = [&](int c) -> int {
        if (P->dry) return ERGM_OK;
        const int b0 = bsplit[c], nb = bsplit[c + 1] - b0;
        const size_t r0 = (size_t)b0 * S;
        const ergm_dropout de = resid_drop(P, 0, b0);  // embedding dropout (src/model.py:506)
        return embed_fwd_ld(P->ids + r0, P->tt ? P->tt + r0 : nullptr, P->cap_ids + r0, p.wte, p.wpe,
                            vis_in ? vis_in + (size_t)b0 * ld_vis : nullptr, ld_vis,
                            aud_in ? aud_in + (size_t)b0 * E : nullptr, P->resid[0] + r0 * E, P->cap + r0 * P->XE,
                            P->XE, nb, S, E, d.vocab, cs[c], drop_site_of(&de, E));
    };
    if (nchain >= 2 && !P->dry) {
        if (hipEventRecord(P->ev_f2[0], s) != hipSuccess) return fail(ERGM_EHIP, "model: chain fork");
        for (int c = 1; c < nchain; ++c) {
            if (hipStreamWaitEvent(cs[c], P->ev_f2[0], 0) != hipSuccess) return fail(ERGM_EHIP, "model: chain fork");
            ERGM_TRY(embed(c));
            if (hipEventRecord(ev_emb[c], cs[c]) != hipSuccess) return fail(ERGM_EHIP, "model: event record");
        }
    }
    ERGM_TRY(embed(0));
    // The cross-attention K/V projections of the caption embeddings, on the side stream (they overlap the chains'
    // first sub-blocks).  kv_per_block: one GEMM per block, in block order, each marked (ev_kv[l]) for that block's
    // cross-attention — block 0 waits for 1/L of the projection instead of all of it (the single 2048 x 18432 x 768
    // GEMM ran alone for ~80 us at C2 while both chains waited, profiles/r06a_timeline.txt) and the rest overlaps the
    // latency-bound forward's idle CUs (+1.7 % per step at C2, profiles/r06_ab_kv.txt).  Otherwise one GEMM for all
    // blocks, joined (side_mark(L)) before block 0's cross-attention.
    {
        ERGM_TRY(fork_side(P, s));
        hipStream_t ss = P->dry ? s : P->side;
        for (int c = 1; c < nchain && !P->dry; ++c)  // the caption rows of every chain are embedded
            if (hipStreamWaitEvent(ss, ev_emb[c], 0) != hipSuccess) return fail(ERGM_EHIP, "model: stream wait");
        if (P->f8) ERGM_TRY(quant_layer_weights(P, 0, ss));
        if (P->f8 && !P->dry) {
            if (P->mx) {
                MxJobs J{};
                J.n = 1;
                J.j[0] = MxJob{reinterpret_cast<const __bf16*>(p.capkv_w_b), P->capkv8, P->capkv8_x, L2E, E, L2E, E,
                               L2E, 0};
                ERGM_TRY(quant_weights_mx(J, ss));
            } else {
                if (hipMemsetAsync(P->capkv_amax, 0, (size_t)L2E * 4, ss) != hipSuccess) return fail(ERGM_EHIP, "memset");
                WqJobs J{};
                J.n = 1;
                J.j[0] = WqJob{p.capkv_w_b, P->capkv8, P->capkv8_s, P->capkv_amax, L2E, E, L2E, E, 0, 0, 1};
                ERGM_TRY(quant_weights_fp8(J, ss));
            }
            ERGM_TRY(quant_act(P, P->cap, P->XE, T, E, P->qcap, P->scap, P->xcap, ss));
        }
    }
    hipStream_t ss = P->dry ? s : P->side;
    // fp8: block l's weights are re-quantised on the side stream too (its forward waits for ev_wq[l]); a deferred
    // AdamW update of block l (FusedAdamW(defer=True)) writes the bf16 shadow the quantiser reads, so the side
    // stream waits for it like block l's forward does
    auto quant_block = [&](int l) -> int {
        if (!P->f8 || l <= 0 || l >= L) return ERGM_OK;
        ERGM_TRY(wait_update(P, l, ss));
        return quant_layer_weights(P, l, ss);
    };
    // the side stream's tail of forward work: the embedding backward's sort (it needs only the ids: done here, off
    // the critical chain), then the mark
    auto side_tail = [&]() -> int {
        if (train && !P->dry)
            ERGM_TRY(embed_bwd_sort(P->ids, P->tt, P->cap_ids, T, d.vocab, P->keys, P->row_flag, d.vocab_pad, ss));
        return side_mark(P, L);
    };
    const bool kvb = P->kv_per_block && !P->dry;
    // block l's caption K/V (+ block l+1's fp8 weights); enqueued one block ahead of its cross-attention, between the
    // chains' launches, so the host reaches the chains' first kernels without enqueuing all L projections first
    auto kv_block = [&](int l) -> int {
        const size_t c0 = (size_t)l * 2 * E;
        if (P->f8)  // rows c0.. of the [L2E][E] weight copy and of its scales (MX pitch: all L2E rows)
            ERGM_TRY(gemm8(P, ss, T, 2 * E, E, P->qcap, P->scap, P->xcap, P->capkv8 + c0 * E,
                           P->capkv8_s ? P->capkv8_s + c0 : nullptr, P->capkv8_x ? P->capkv8_x + c0 * 4 : nullptr,
                           P->kv_all + c0, L2E, ERGM_BF16, ERGM_EPI_BIAS, p.capkv_b + c0, nullptr, 0, nullptr, 0,
                           nullptr, nullptr, nullptr, L2E));
        else
            ERGM_TRY(gemm(P, ss, T, 2 * E, E, P->cap, P->XE, ERGM_MK, reinterpret_cast<const __bf16*>(p.capkv_w_b) + c0,
                          L2E, ERGM_KN, P->kv_all + c0, L2E, ERGM_BF16, ERGM_EPI_BIAS, p.capkv_b + c0));
        if (hipEventRecord(P->ev_kv[l], ss) != hipSuccess) return fail(ERGM_EHIP, "model: event record");
        ERGM_TRY(quant_block(l + 1));  // block l+1's weights before block l+1's K/V (its forward needs both)
        return l == L - 1 ? side_tail() : ERGM_OK;
    };
    if (kvb) {
        ERGM_TRY(kv_block(0));
    } else {
        {
            Probe pr(P, 4, ss);
            if (P->f8)
                ERGM_TRY(gemm8(P, ss, T, L2E, E, P->qcap, P->scap, P->xcap, P->capkv8, P->capkv8_s, P->capkv8_x,
                               P->kv_all, L2E, ERGM_BF16, ERGM_EPI_BIAS, p.capkv_b));
            else
                ERGM_TRY(gemm(P, ss, T, L2E, E, P->cap, P->XE, ERGM_MK, p.capkv_w_b, L2E, ERGM_KN, P->kv_all, L2E,
                              ERGM_BF16, ERGM_EPI_BIAS, p.capkv_b));
        }
        ERGM_TRY(side_tail());
        for (int l = 1; l < L; ++l) ERGM_TRY(quant_block(l));
    }
    // Enqueue order: launch by launch, alternating chains.  The forward's kernels are short, so the host's enqueue
    // pace can set the GPU's: enqueued a block at a time, the chains ran one block after the other instead of side
    // by side (profiles/r01_overlap_experiments.txt).
    constexpr int NP = 11;  // fwd_block parts
    for (int g = 0; g < L * NP; ++g) {
        if (kvb && g % NP == 1 && g / NP + 1 < L) ERGM_TRY(kv_block(g / NP + 1));
        for (int c = 0; c < nchain; ++c) ERGM_TRY(fwd_block(P, g / NP, cs[c], bsplit[c], bsplit[c + 1] - bsplit[c], g % NP));
    }
    for (int c = 1; c < nchain && !P->dry; ++c)
        if (hipEventRecord(ev_done[c], cs[c]) != hipSuccess || hipStreamWaitEvent(s, ev_done[c], 0) != hipSuccess)
            return fail(ERGM_EHIP, "model: chain join");
    // every stream's forward work joined into the caller's stream (the side stream's tail — the embedding backward's
    // sort — long done by now; a captured forward must not leave it unjoined)
    if (kvb) ERGM_TRY(join_side(P, s, L));
    if (!P->dry)
        ERGM_TRY(ergm_layernorm_fwd(P->resid[3 * L], p.ln_f_w, p.ln_f_b, P->lnf, P->mf, P->rf, T, E, d.eps, s));
    // tied LM head: logits = ln_f(h) · wteᵀ over the padded vocab (pad rows of wte are zero)
    {
        const int n0 = lmhead_split_cols(T, d.vocab_pad);
        {
            Probe pr(P, 1, s);  // the bench's roofline kernel: the whole-round main launch
            ERGM_TRY(gemm(P, s, T, n0, E, P->lnf, E, ERGM_MK, p.wte_b, E, ERGM_NK, logits, d.vocab_pad,
                          ERGM_BF16, ERGM_EPI_NONE));
        }
        if (n0 < d.vocab_pad)
            ERGM_TRY(gemm(P, s, T, d.vocab_pad - n0, E, P->lnf, E, ERGM_MK,
                          reinterpret_cast<const __bf16*>(p.wte_b) + (size_t)n0 * E, E, ERGM_NK,
                          reinterpret_cast<__bf16*>(logits) + n0, d.vocab_pad, ERGM_BF16, ERGM_EPI_NONE));
    }
    if (P->dry) return ERGM_OK;
    ERGM_TRY(ergm_emotion_head(P->lnf, p.emo_w, P->emo_labels, emo_logits, P->emo_sum, nullptr, nullptr, P->emo_tmp,
                               B, S, E, 7, P->n_valid ? P->n_valid + 1 : nullptr, nullptr, s));
    if (P->labels) {
        ERGM_TRY(ergm_xent_fwd_bwd(logits, d.vocab_pad, P->labels, P->n_valid, P->row_loss, train ? P->dlogits : nullptr,
                                   B, S, d.vocab, 1.0f, s));
    } else if (train) {
        ERGM_TRY(hipMemsetAsync(P->dlogits, 0, (size_t)T * d.vocab_pad * 2, s) == hipSuccess ? ERGM_OK : ERGM_EHIP);
        ERGM_TRY(hipMemsetAsync(P->row_loss, 0, (size_t)T * 4, s) == hipSuccess ? ERGM_OK : ERGM_EHIP);
    }
    if (P->labels || P->emo_labels) {
        if (!P->labels) ERGM_TRY(hipMemsetAsync(P->row_loss, 0, (size_t)T * 4, s) == hipSuccess ? ERGM_OK : ERGM_EHIP);
        if (train && (P->metric_loss || P->metric_correct))
            ERGM_TRY(loss_finalize_metrics(P->row_loss, T, P->labels ? P->n_valid : nullptr,
                                           P->emo_labels ? P->emo_sum : nullptr, P->n_valid + 1, out_loss,
                                           P->metric_loss, P->emo_labels ? P->metric_correct : nullptr, emo_logits,
                                           P->emo_labels, B, 7, s));
        else
            ERGM_TRY(ergm_loss_finalize(P->row_loss, T, P->labels ? P->n_valid : nullptr,
                                        P->emo_labels ? P->emo_sum : nullptr, P->n_valid + 1, out_loss, s));
    }
    P->have_fwd = train != 0;
    if (!P->dry)
        for (auto& f : P->upd_pending) f = 0;  // every block's forward waited for its update
    return check_launch("model_forward");
}

}  // namespace

extern "C" int ergm_model_forward(ergm_model_plan* P, void* logits, float* emo_logits, float* out_loss, int train,
                                  void* stream) {
    ERGM_CHECK_ARG(P && logits && emo_logits, "model_forward: null argument");
    ERGM_CHECK_ARG(P->ids, "model_forward: call ergm_model_set_inputs first");
    ERGM_CHECK_ARG(!(P->labels || P->emo_labels) || out_loss, "model_forward: labels need out_loss");
    bind_clear();
    P->stage_pt = nullptr;  // a fork point is armed and taken inside one native call
    hipStream_t s = as_stream(stream);
    if (P->ones_pending) {  // before any fork from s: every other stream of the step is ordered after these
        const ergm_model_dims& d = P->d;
        for (int l = 0; l < d.n_layer; ++l) {
            LayerActs& a = P->la[l];
            const void* cols[5] = {a.ln1, a.lnx, a.ln2, a.ao, a.xo};
            for (int i = 0; i < 5; ++i) ERGM_TRY(fill_ones_col((void*)cols[i], P->T, P->XE, d.n_embd, s));
            ERGM_TRY(fill_ones_col(a.act, P->T, P->XF, d.n_inner, s));
        }
        ERGM_TRY(fill_ones_col(P->cap, P->T, P->XE, d.n_embd, s));
        P->ones_pending = false;
    }
    return do_forward(P, logits, emo_logits, out_loss, train, s);
}

namespace {

int do_backward_head(ergm_model_plan* P, const float* gscale, hipStream_t s) {
    const ergm_model_dims& d = P->d;
    P->ln_pending = 0;
    P->bwd_forked = false;
    const ergm_model_params& p = P->p;
    const int T = P->T, E = d.n_embd, B = d.batch, S = d.seq, Vp = d.vocab_pad, L = d.n_layer;
    // dh_f = dlogits · wte (contraction over the padded vocab) on the main chain; the tied-weight
    // gradient dwte = dlogitsᵀ · ln_f(h) on the side stream (joined before the embedding backward adds
    // the lookup gradients into the same buffer).
    // a caller's gradient on the returned logits (src/model.py:698 returns differentiable logits): added to the
    // cross-entropy's dlogits, scaled by the loss gradient there, so the LM-head GEMMs run with alpha 1
    const float* lm_scale = gscale;
    if (P->logits_grad && !P->dry) {
        ERGM_TRY(dlogits_add(P->dlogits, P->logits_grad, gscale, (size_t)T * Vp, s));
        lm_scale = nullptr;
    }
    P->logits_grad = nullptr;
    auto lm_dw = [&]() -> int {
        ERGM_TRY(fork_side(P, s));
        hipStream_t ss = P->dry ? s : P->side;
        Probe pr(P, 3, ss);
        Probe pr5(P, 5, ss, 2.0 * Vp * E * T);
        ERGM_TRY(gemm(P, ss, Vp, E, T, P->dlogits, Vp, ERGM_KM, P->lnf, E, ERGM_KN, p.g_wte, E, ERGM_F32,
                      ERGM_EPI_NONE, nullptr, nullptr, 0, nullptr, 0, lm_scale));
        return side_mark(P, L + 1);
    };
    if (P->lm_dw_first) ERGM_TRY(lm_dw());
    {
        Probe pr(P, 2, s);
        ERGM_TRY(gemm(P, s, T, E, Vp, P->dlogits, Vp, ERGM_MK, p.wte_b, E, ERGM_KN, P->dy, E, ERGM_F32, ERGM_EPI_NONE,
                      nullptr, nullptr, 0, nullptr, 0, lm_scale));
    }
    if (!P->lm_dw_first) ERGM_TRY(lm_dw());
    if (P->dry) return ERGM_OK;
    if (P->emo_labels) {
        ERGM_TRY(ergm_emotion_head(P->lnf, p.emo_w, P->emo_labels, P->emo_tmp, P->emo_tmp + (size_t)B * 7, p.g_emo_w,
                                   P->dy, P->emo_tmp + (size_t)B * 8 + 4, B, S, E, 7, P->n_valid + 1, gscale, s));
    } else {
        if (hipMemsetAsync(p.g_emo_w, 0, (size_t)7 * E * 4, s) != hipSuccess) return fail(ERGM_EHIP, "memset");
    }
    if (hipMemsetAsync(P->dh, 0, (size_t)T * E * 4, s) != hipSuccess) return fail(ERGM_EHIP, "memset");
    return ln_bwd(P, s, P->resid[3 * L], P->mf, P->rf, p.ln_f_w, p.g_ln_f_w, p.g_ln_f_b, P->dhb[3 * L], 3 * L);
}

// The fused attention backward (dO GEMM inside) runs one 512-thread workgroup per (sample, head); with more of them
// than the chip has CUs its GEMM part runs in rounds and the form loses to the two launches (C5, B·H = 512: -2.5 %;
// C2, 192: level, profiles/r04_experiments.txt #12).
constexpr int kAttnFuseMaxWg = 256;

int do_backward_layer(ergm_model_plan* P, int l, hipStream_t s) {
    const ergm_model_dims& d = P->d;
    const int E = d.n_embd, F = d.n_inner, H = d.n_head, S = d.seq, L2E = P->L2E;
    const int L = d.n_layer;
    const Chains ch = bwd_chains(P, s);
    if (ch.n == 2 && !P->bwd_forked) {  // the second chain starts from the head stage's outputs
        if (hipEventRecord(P->ev_f2[0], s) != hipSuccess || hipStreamWaitEvent(P->fwd2, P->ev_f2[0], 0) != hipSuccess)
            return fail(ERGM_EHIP, "model: backward chain fork");
        P->bwd_forked = true;
    }
    LayerActs a = P->dry ? LayerActs{} : P->la[l];
    const float* x0 = P->dry ? nullptr : P->resid[3 * l];
    const float* x1 = P->dry ? nullptr : P->resid[3 * l + 1];
    const float* x2 = P->dry ? nullptr : P->resid[3 * l + 2];
    __bf16* dh3 = P->dhb[3 * l + 3];  // bf16 grad of this block's output (written by the previous stage)
    __bf16* dh2 = P->dhb[3 * l + 2];
    __bf16* dh1 = P->dhb[3 * l + 1];
    __bf16* dh0 = P->dhb[3 * l];
    __bf16* dpre = P->dpre[l];
    __bf16* dxq = P->dxq[l];
    __bf16* dqkv = P->dqkv[l];
    // per-chain row offset helper (dry run: pointers stay null)
    auto R = [&](auto* p, int c, size_t ld) { return (P->dry || !p) ? p : p + (size_t)ch.b0[c] * S * ld; };
    auto Tc = [&](int c) { return ch.nb[c] * S; };
    // the block LayerNorms' incoming gradient (ln_bwd_rows reads the same buffer): bf16, or f32 (ln_dy_f32)
    auto DYO = [&](int c) { return P->ln_dy_f32 ? (void*)R(P->dy, c, E) : (void*)R(P->dyb, c, E); };
    const int dyo_t = P->ln_dy_f32 ? ERGM_F32 : ERGM_BF16;
    // Weight-gradient pairs (mlp c_proj + c_fc, cross c_proj + q, attn c_proj + c_attn) are forked to the side
    // stream once the dY of the second member is formed.
    // fork points: with one data-gradient chain, the launch each weight-gradient fork waits for carries the
    // fork's event itself (arm_fork before it) instead of a marker packet recorded behind it
    const bool arm = ch.n == 1 && !P->dry;
    // ---- MLP: x3 = x2 + drop(gelu(ln2(x2)·Wfc + bfc)·Wm + bm)
    ERGM_TRY(dw_gemm(P, ch, F, E, a.act, P->XF, dh3, E, LG(P, l, ERGM_T_MPROJ_W), LG(P, l, ERGM_T_MPROJ_B)));
    if (arm) arm_fork(P, s);  // dpre (mlp c_proj dX with GELU'): the c_fc dW's dY
    for (int c = 0; c < ch.n; ++c)
        ERGM_TRY(gemm(P, ch.s[c], Tc(c), F, E, R(dh3, c, E), E, ERGM_MK, LB(P, l, ERGM_T_MPROJ_W), E, ERGM_NK,
                      R(dpre, c, F), F, ERGM_BF16, ERGM_EPI_GELU_BWD, nullptr, R(a.pre, c, F), F));
    ERGM_TRY(dw_gemm(P, ch, E, F, a.ln2, P->XE, dpre, F, LG(P, l, ERGM_T_FC_W), LG(P, l, ERGM_T_FC_B)));
    ERGM_TRY(dw_flush(P, ch));  // mlp c_proj + c_fc weight gradients
    for (int c = 0; c < ch.n; ++c)
        ERGM_TRY(gemm(P, ch.s[c], Tc(c), E, F, R(dpre, c, F), F, ERGM_MK, LB(P, l, ERGM_T_FC_W), F, ERGM_NK,
                      DYO(c), E, dyo_t, ERGM_EPI_NONE));
    for (int c = 0; c < ch.n; ++c)
        ERGM_TRY(ln_bwd_rows(P, ch.s[c], x2, a.m2, a.r2, LF(P, l, ERGM_T_LN2_W), dh2, 3 * l + 2, ch.b0[c] * S, Tc(c)));
    ERGM_TRY(ln_reduce_add(P, 3 * l + 2, LG(P, l, ERGM_T_LN2_W), LG(P, l, ERGM_T_LN2_B)));
    // ---- cross-attention: x2 = x1 + drop(Attn(ln_x(x1)·Wq + bq, KV_l(cap))·Wxp + bxp)
    ERGM_TRY(dw_gemm(P, ch, E, E, a.xo, P->XE, dh2, E, LG(P, l, ERGM_T_XPROJ_W), LG(P, l, ERGM_T_XPROJ_B)));
    for (int c = 0; c < ch.n; ++c) {
        if (P->attn_fuse && ch.nb[c] * H <= kAttnFuseMaxWg) {  // dO = dh2·Wxpᵀ formed inside the attention backward
            if (arm) arm_fork(P, s);  // the cross-attention backward: dxq, the q dW's dY
            if (!P->dry) {
                const __bf16* kl = R(P->kv_all, c, L2E) + (size_t)l * 2 * E;
                __bf16* dkl = R(P->dkv_all, c, L2E) + (size_t)l * 2 * E;
                const ergm_dropout dp = attn_drop(P, l, 1, ch.b0[c]);
                const size_t bhs = (size_t)ch.b0[c] * H * S;
                ERGM_TRY(attn_bwd_fused(R(a.xq, c, E), kl, kl + E, R(a.xo, c, P->XE), R(dh2, c, E), E,
                                        LB(P, l, ERGM_T_XPROJ_W), E, E, a.xlse + bhs, R(dxq, c, E), dkl, dkl + E,
                                        ch.nb[c], H, S, S, E, L2E, L2E, P->XE, E, L2E, L2E, 0, &dp,
                                        attn_bits(P, l, 1, ch.b0[c]), ch.s[c]));
            }
            continue;
        }
        ERGM_TRY(gemm(P, ch.s[c], Tc(c), E, E, R(dh2, c, E), E, ERGM_MK, LB(P, l, ERGM_T_XPROJ_W), E, ERGM_NK,
                      R(P->d_o, c, E), E, ERGM_BF16, ERGM_EPI_NONE));
        if (arm) arm_fork(P, s);  // the cross-attention backward: dxq, the q dW's dY
        if (!P->dry) {
            const __bf16* kl = R(P->kv_all, c, L2E) + (size_t)l * 2 * E;
            __bf16* dkl = R(P->dkv_all, c, L2E) + (size_t)l * 2 * E;
            const ergm_dropout dp = attn_drop(P, l, 1, ch.b0[c]);
            const size_t bhs = (size_t)ch.b0[c] * H * S;
            ERGM_TRY(ergm_attn_bwd(R(a.xq, c, E), kl, kl + E, R(a.xo, c, P->XE), R(P->d_o, c, E), a.xlse + bhs,
                                   P->delta + bhs, R(dxq, c, E), dkl, dkl + E, ch.nb[c], H, S, S, E, L2E, L2E, P->XE,
                                   E, E, L2E, L2E, 0, &dp, attn_bits(P, l, 1, ch.b0[c]), ch.s[c]));
        }
    }
    ERGM_TRY(dw_gemm(P, ch, E, E, a.lnx, P->XE, dxq, E, LG(P, l, ERGM_T_XQ_W), LG(P, l, ERGM_T_XQ_B)));
    ERGM_TRY(dw_flush(P, ch));  // cross c_proj + q weight gradients
    for (int c = 0; c < ch.n; ++c)
        ERGM_TRY(gemm(P, ch.s[c], Tc(c), E, E, R(dxq, c, E), E, ERGM_MK, LB(P, l, ERGM_T_XQ_W), E, ERGM_NK,
                      DYO(c), E, dyo_t, ERGM_EPI_NONE));
    for (int c = 0; c < ch.n; ++c)
        ERGM_TRY(ln_bwd_rows(P, ch.s[c], x1, a.mx, a.rx, LF(P, l, ERGM_T_LNX_W), dh1, 3 * l + 1, ch.b0[c] * S, Tc(c)));
    ERGM_TRY(ln_reduce_add(P, 3 * l + 1, LG(P, l, ERGM_T_LNX_W), LG(P, l, ERGM_T_LNX_B)));
    // ---- self-attention: x1 = x0 + drop(Attn(ln_1(x0)·Wqkv + b)·Wap + bap)
    ERGM_TRY(dw_gemm(P, ch, E, E, a.ao, P->XE, dh1, E, LG(P, l, ERGM_T_APROJ_W), LG(P, l, ERGM_T_APROJ_B)));
    for (int c = 0; c < ch.n; ++c) {
        if (P->attn_fuse && ch.nb[c] * H <= kAttnFuseMaxWg) {  // dO = dh1·Wapᵀ formed inside the attention backward
            if (arm) arm_fork(P, s);  // the self-attention backward: dqkv, the c_attn dW's dY
            if (!P->dry) {
                const ergm_dropout dp = attn_drop(P, l, 0, ch.b0[c]);
                const size_t bhs = (size_t)ch.b0[c] * H * S;
                const __bf16* q = R(a.qkv, c, 3 * E);
                __bf16* dq = R(dqkv, c, 3 * E);
                ERGM_TRY(attn_bwd_fused(q, q + E, q + 2 * E, R(a.ao, c, P->XE), R(dh1, c, E), E,
                                        LB(P, l, ERGM_T_APROJ_W), E, E, a.lse + bhs, dq, dq + E, dq + 2 * E, ch.nb[c],
                                        H, S, S, 3 * E, 3 * E, 3 * E, P->XE, 3 * E, 3 * E, 3 * E, 1, &dp,
                                        attn_bits(P, l, 0, ch.b0[c]), ch.s[c]));
            }
            continue;
        }
        ERGM_TRY(gemm(P, ch.s[c], Tc(c), E, E, R(dh1, c, E), E, ERGM_MK, LB(P, l, ERGM_T_APROJ_W), E, ERGM_NK,
                      R(P->d_o, c, E), E, ERGM_BF16, ERGM_EPI_NONE));
        if (arm) arm_fork(P, s);  // the self-attention backward: dqkv, the c_attn dW's dY
        if (!P->dry) {
            const ergm_dropout dp = attn_drop(P, l, 0, ch.b0[c]);
            const size_t bhs = (size_t)ch.b0[c] * H * S;
            const __bf16* q = R(a.qkv, c, 3 * E);
            __bf16* dq = R(dqkv, c, 3 * E);
            ERGM_TRY(ergm_attn_bwd(q, q + E, q + 2 * E, R(a.ao, c, P->XE), R(P->d_o, c, E), a.lse + bhs, P->delta + bhs,
                                   dq, dq + E, dq + 2 * E, ch.nb[c], H, S, S, 3 * E, 3 * E, 3 * E, P->XE, E, 3 * E,
                                   3 * E, 3 * E, 1, &dp, attn_bits(P, l, 0, ch.b0[c]), ch.s[c]));
        }
    }
    ERGM_TRY(dw_gemm(P, ch, E, 3 * E, a.ln1, P->XE, dqkv, 3 * E, LG(P, l, ERGM_T_ATTN_W), LG(P, l, ERGM_T_ATTN_B)));
    ERGM_TRY(dw_flush(P, ch));  // attn c_proj + c_attn weight gradients
    for (int c = 0; c < ch.n; ++c)
        ERGM_TRY(gemm(P, ch.s[c], Tc(c), E, 3 * E, R(dqkv, c, 3 * E), 3 * E, ERGM_MK, LB(P, l, ERGM_T_ATTN_W), 3 * E,
                      ERGM_NK, DYO(c), E, dyo_t, ERGM_EPI_NONE));
    for (int c = 0; c < ch.n; ++c) {
        if (arm) arm_fork(P, s);  // ln_1's backward: the stage's last launch (LayerNorm reduce, optimizer)
        ERGM_TRY(ln_bwd_rows(P, ch.s[c], x0, a.m1, a.r1, LF(P, l, ERGM_T_LN1_W), dh0, 3 * l, ch.b0[c] * S, Tc(c)));
    }
    ERGM_TRY(ln_reduce_add(P, 3 * l, LG(P, l, ERGM_T_LN1_W), LG(P, l, ERGM_T_LN1_B)));
    // side-stream dW GEMMs of this block are marked; the caller's stream waits (one block late) for
    // those of the block differentiated before, so block l+1's gradients are final on return.
    ERGM_TRY(ln_reduce_flush(P, ch));  // this block's three LayerNorms (+ ln_f after the head stage)
    ERGM_TRY(side_mark(P, l));
    if (l + 1 < L && P->per_stage_join) ERGM_TRY(join_side(P, s, l + 1));
    return ERGM_OK;
}

int do_backward_embed(ergm_model_plan* P, hipStream_t s) {
    const ergm_model_dims& d = P->d;
    const ergm_model_params& p = P->p;
    const int T = P->T, E = d.n_embd, L2E = P->L2E, L = d.n_layer;
    if (P->bwd_forked) {  // the second backward chain's rows of dh are final: join it
        if (hipEventRecord(P->ev_f2[2], P->fwd2) != hipSuccess || hipStreamWaitEvent(s, P->ev_f2[2], 0) != hipSuccess)
            return fail(ERGM_EHIP, "model: backward chain join");
        P->bwd_forked = false;
    }
    // dh is already the gradient of the embedding sum: block 0's first LayerNorm backward took it through
    // the embedding dropout (ln_bwd_rows, slot 0)
    if (P->proj) {
        // feature projections: the projected vectors got dh0 at positions 0 / 1; dW = featᵀ·d over the
        // (padded) batch with the bias row fused (side stream); no gradient flows to the features
        const int Fd = P->Fd, Bp = P->Bp, ldf = P->Fd + 8;
        if (P->dry || P->vis) {
            if (!P->dry) ERGM_TRY(proj_grad_pack(P->dh, P->dproj, d.batch, Bp, d.seq, E, s));
            ERGM_TRY(fork_side(P, s));
            hipStream_t ss = P->dry ? s : P->side;
            for (int m = 0; m < 2; ++m) {
                float* gw = m == 0 ? p.g_vproj_w : p.g_aproj_w;
                ERGM_TRY(gemm(P, ss, Fd + 1, E, Bp, P->feat_b16 ? P->feat_b16 + (size_t)m * Bp * ldf : nullptr, ldf,
                              ERGM_KM, P->dproj ? P->dproj + (size_t)m * Bp * E : nullptr, E, ERGM_KN, gw, E, ERGM_F32,
                              ERGM_EPI_NONE));
            }
        } else {  // text-only batch through a projected model: zero projection gradients
            const size_t n = ((size_t)Fd + 1) * E * sizeof(float);
            if (hipMemsetAsync(p.g_vproj_w, 0, n, s) != hipSuccess || hipMemsetAsync(p.g_aproj_w, 0, n, s) != hipSuccess)
                return fail(ERGM_EHIP, "model: memset");
        }
    }
    {  // the stacked caption K/V projection: dW = capᵀ·dKV_all (side), dcap = dKV_all·Wᵀ (main), one GEMM each
        // (per block instead, in the block stages: 0.25 ms/step slower at C2, profiles/r03_experiments.txt #6)
        const Chains one{1, {s, s}, {0, 0}, {d.batch, 0}};
        ERGM_TRY(dw_gemm(P, one, E, L2E, P->cap, P->XE, P->dkv_all, L2E, p.g_capkv_w, p.g_capkv_b));
        ERGM_TRY(dw_flush(P, one));
        ERGM_TRY(gemm(P, s, T, E, L2E, P->dkv_all, L2E, ERGM_MK, p.capkv_w_b, L2E, ERGM_NK, P->dcap, E, ERGM_F32,
                      ERGM_EPI_NONE));
    }
    // mark the side stream's caption / projection work
    ERGM_TRY(side_mark(P, L + 2));
    if (P->dry) return ERGM_OK;
    // the LM-head dwte (side stream, marked L+1) is final before the lookup gradients are added to it;
    // the caption K/V weight gradient keeps running on the side stream meanwhile
    ERGM_TRY(join_side(P, s, L + 1));
    ERGM_TRY(ws_need(P, (size_t)3 * T * E * sizeof(float)));
    ERGM_TRY(embed_bwd_sums(P->keys, d.batch, d.seq, E, P->dh, P->dcap,
                            P->lookup_compact ? P->lookup_compact : p.g_wte, p.g_wpe,
                            reinterpret_cast<float*>(P->scratch), P->lookup_compact ? P->row_pos : nullptr, s));
    return join_side(P, s, L + 2);  // every gradient final on the caller's stream
}

}  // namespace

extern "C" int ergm_model_set_optimizer(ergm_model_plan* P, const ergm_adamw_desc* o) {
    ERGM_CHECK_ARG(P, "model_set_optimizer: null plan");
    if (!o) {
        P->opt_on = false;
        return ERGM_OK;
    }
    const int L = P->d.n_layer;
    ERGM_CHECK_ARG(o->param && o->grad && o->exp_avg && o->exp_avg_sq && o->ranges && o->n_ranges == L + 1,
                   "model_set_optimizer: null buffer or n_ranges != n_layer + 1");
    for (int k = 0; k <= L; ++k)
        ERGM_CHECK_ARG(o->ranges[2 * k] >= 0 && o->ranges[2 * k + 1] > o->ranges[2 * k] &&
                           o->ranges[2 * k] % 4 == 0 && o->ranges[2 * k + 1] % 4 == 0,
                       "model_set_optimizer: range %d must be non-empty, 4-element aligned", k);
    ERGM_CHECK_ARG(o->wte_begin >= 0 && o->wte_begin % 4 == 0, "model_set_optimizer: bad wte_begin");
    if (!P->opt_s) {
        if (make_stream(&P->opt_s) != hipSuccess)
            return fail(ERGM_EHIP, "model_set_optimizer: stream creation");
        P->ev_opt.assign(L + 4, nullptr);
        for (auto& e : P->ev_opt)
            if (hipEventCreateWithFlags(&e, kSyncEv) != hipSuccess) return fail(ERGM_EHIP, "model_set_optimizer: event");
        P->ev_upd.assign(L, nullptr);
        for (auto& e : P->ev_upd)
            if (hipEventCreateWithFlags(&e, kSyncEv) != hipSuccess) return fail(ERGM_EHIP, "model_set_optimizer: event");
        P->upd_pending.assign(L, 0);
    }
    P->opt = *o;
    P->opt_ranges.assign(o->ranges, o->ranges + 2 * (L + 1));
    P->opt.ranges = P->opt_ranges.data();
    P->opt_on = true;
    return ERGM_OK;
}

namespace {
// The optimizer stream waits for everything issued so far on `s` — the stage just enqueued, so a bucket's update
// launched `lag` stages after its block overlaps the later blocks (opt_after_layer) — and, for mark >= 0, for the side
// stream's weight-gradient mark of that stage (its gradients).  The point on `s` is the stage's final fork point
// taken in this same native call (ln_reduce_flush: nothing has been enqueued on s since), else a fresh event.
int opt_wait(ergm_model_plan* P, hipStream_t s, int mark) {
    hipEvent_t e = P->stage_pt;
    if (!e) {
        e = P->ev_opt[P->opt_k++ % P->ev_opt.size()];
        if (hipEventRecord(e, s) != hipSuccess) return fail(ERGM_EHIP, "model: optimizer stream wait");
    }
    if (hipStreamWaitEvent(P->opt_s, e, 0) != hipSuccess) return fail(ERGM_EHIP, "model: optimizer stream wait");
    if (mark >= 0 && hipStreamWaitEvent(P->opt_s, P->ev_join[mark], 0) != hipSuccess)
        return fail(ERGM_EHIP, "model: optimizer stream wait");
    return ERGM_OK;
}
int opt_range(ergm_model_plan* P, int64_t a, int64_t b) {
    const ergm_adamw_desc& o = P->opt;
    void* sh = o.param_bf16 ? reinterpret_cast<__bf16*>(o.param_bf16) + a : nullptr;
    return ergm_adamw_step(o.param + a, o.grad + a, o.exp_avg + a, o.exp_avg_sq + a, sh, (size_t)(b - a), o.lr, o.beta1,
                           o.beta2, o.eps, o.weight_decay, o.step_size, o.bc2_sqrt, o.max_blocks, P->opt_s);
}
int opt_wte(ergm_model_plan* P, int select) {  // the tied wte's untouched (0) / touched (1) rows
    const ergm_adamw_desc& o = P->opt;
    const int64_t a = o.wte_begin, E = P->d.n_embd, rows = P->d.vocab_pad;
    if (!P->row_flag) return select ? opt_range(P, a, a + rows * E) : ERGM_OK;
    void* sh = o.param_bf16 ? reinterpret_cast<__bf16*>(o.param_bf16) + a : nullptr;
    return ergm_adamw_rows(o.param + a, o.grad + a, o.exp_avg + a, o.exp_avg_sq + a, sh, (int)rows, (int)E, P->row_flag,
                           select, o.lr, o.beta1, o.beta2, o.eps, o.weight_decay, o.step_size, o.bc2_sqrt, o.max_blocks,
                           P->opt_s);
}
int opt_after_layer(ergm_model_plan* P, int l, hipStream_t s) {
    if (!P->opt_on || P->dry) return ERGM_OK;
    const int L = P->d.n_layer, i = L - 1 - l;
    // Block m's bucket (L-1-m) is final with its weight-gradient mark m (recorded after the LayerNorm reduce,
    // which waited for the stage's last LayerNorm backward, so the stage has read the old weights).  Its AdamW
    // is launched `lag` stages later (opt_lag = 2): the update then overlaps later blocks' backward
    // instead of competing with its own block's weight-gradient GEMMs (bench A/B: lag 2 vs 1 C2 -0.4 %, C5
    // -0.6 %, C4 equal; lag 0 slower).
    const int lag = P->opt_lag;
    auto upd = [&](int m) -> int {
        ERGM_TRY(opt_wait(P, s, m));
        return opt_range(P, P->opt.ranges[2 * (L - 1 - m)], P->opt.ranges[2 * (L - 1 - m) + 1]);
    };
    if (!P->opt.defer) {
        if (l + lag <= L - 1) ERGM_TRY(upd(l + lag));
        if (l == 0)  // the remaining blocks, last stage first
            for (int m = std::min(lag, L) - 1; m >= 0; --m) ERGM_TRY(upd(m));
    }
    if (i == std::min(1, L - 1) && !(L == 1 && lag >= 1)) {  // the LM-head part of the tied wte (mark L+1)
        ERGM_TRY(opt_wait(P, s, L + 1));
        ERGM_TRY(opt_wte(P, 0));
    }
    return ERGM_OK;
}
int opt_after_embed(ergm_model_plan* P, hipStream_t s) {
    if (!P->opt_on || P->dry) return ERGM_OK;
    const int L = P->d.n_layer;
    ERGM_TRY(opt_wait(P, s, -1));  // the embedding stage joined every side-stream gradient
    if (P->opt.defer) ERGM_TRY(opt_range(P, P->opt.ranges[2 * (L - 1)], P->opt.ranges[2 * (L - 1) + 1]));
    if (L == 1 && P->opt_lag >= 1) ERGM_TRY(opt_wte(P, 0));
    ERGM_TRY(opt_range(P, P->opt.ranges[2 * L], P->opt.ranges[2 * L + 1]));
    ERGM_TRY(opt_wte(P, 1));
    hipEvent_t e = P->ev_opt[P->opt_k++ % P->ev_opt.size()];
    if (hipEventRecord(e, P->opt_s) != hipSuccess || hipStreamWaitEvent(s, e, 0) != hipSuccess)
        return fail(ERGM_EHIP, "model: optimizer stream join");
    if (P->opt.defer) {  // blocks 1 … L-1 (bucket L-1-l; bucket 0 also holds the head), in forward order
        for (int l = 1; l < L; ++l) {
            const int i = L - 1 - l;
            ERGM_TRY(opt_range(P, P->opt.ranges[2 * i], P->opt.ranges[2 * i + 1]));
            if (hipEventRecord(P->ev_upd[l], P->opt_s) != hipSuccess) return fail(ERGM_EHIP, "model: event record");
            P->upd_pending[l] = 1;
        }
    }
    return ERGM_OK;
}
// The forward of block l on stream s waits for its deferred update (a no-op unless one is pending).
int wait_update(ergm_model_plan* P, int l, hipStream_t s) {
    if (P->dry || P->upd_pending.empty() || !P->upd_pending[l]) return ERGM_OK;
    return hipStreamWaitEvent(s, P->ev_upd[l], 0) == hipSuccess ? ERGM_OK : fail(ERGM_EHIP, "model: update wait");
}
}  // namespace

extern "C" int ergm_model_optimizer_join(ergm_model_plan* P, void* stream) {
    ERGM_CHECK_ARG(P, "model_optimizer_join: null plan");
    for (size_t l = 0; l < P->upd_pending.size(); ++l)
        if (P->upd_pending[l]) {
            if (hipStreamWaitEvent(as_stream(stream), P->ev_upd[l], 0) != hipSuccess)
                return fail(ERGM_EHIP, "model_optimizer_join: hipStreamWaitEvent");
            P->upd_pending[l] = 0;
        }
    return ERGM_OK;
}

extern "C" int ergm_model_backward_head(ergm_model_plan* P, const float* gscale, void* stream) {
    ERGM_CHECK_ARG(P, "model_backward_head: null plan");
    ERGM_CHECK_ARG(P->have_fwd, "model_backward_head: no training forward to differentiate");
    bind_clear();
    P->stage_pt = nullptr;
    return do_backward_head(P, gscale, as_stream(stream));
}

extern "C" int ergm_model_backward_layer(ergm_model_plan* P, int layer, void* stream) {
    ERGM_CHECK_ARG(P && layer >= 0 && layer < P->d.n_layer, "model_backward_layer: bad layer");
    ERGM_CHECK_ARG(P->have_fwd, "model_backward_layer: no training forward to differentiate");
    bind_clear();
    P->stage_pt = nullptr;
    ERGM_TRY(do_backward_layer(P, layer, as_stream(stream)));
    return opt_after_layer(P, layer, as_stream(stream));
}

extern "C" int ergm_model_backward_embed(ergm_model_plan* P, void* stream) {
    ERGM_CHECK_ARG(P, "model_backward_embed: null plan");
    ERGM_CHECK_ARG(P->have_fwd, "model_backward_embed: no training forward to differentiate");
    bind_clear();
    P->stage_pt = nullptr;
    ERGM_TRY(do_backward_embed(P, as_stream(stream)));
    return opt_after_embed(P, as_stream(stream));
}
