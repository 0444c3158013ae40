// Cross-entropy losses of GPT2LMHeadModel for gfx950.
//
// LM loss: CrossEntropyLoss(ignore_index=-100, mean) on logits[..., :-1, :] vs labels[..., 1:]
// (src/model.py:704-708) — one 512-thread workgroup per logits row keeps the whole bf16 row in
// registers (single HBM read), computes max / Σexp / LSE with one fused block reduction, and writes
// dlogits = (softmax − onehot)/n_valid in the same pass (forward and backward fused; the shift is
// pure indexing: row (b, s) is scored against labels[b][s+1]).
// Emotion loss: emotion_head on the last token + CrossEntropyLoss (src/model.py:700-701,710-711).
#include "common.h"

namespace ergm {

constexpr int XE_THREADS = 512;  // one workgroup per logits row; 8 waves
constexpr int XE_MAXCH = 16;     // 16-B chunks per thread: rows up to 16*512*8 = 65536 columns

// (max, Σexp) pair of online softmax: combine two partial pairs
__device__ __forceinline__ void ms_combine(float& m, float& s, float m2, float s2) {
    const float mn = fmaxf(m, m2);
    if (mn == -INFINITY) return;
    s = s * __expf(m - mn) + s2 * __expf(m2 - mn);
    m = mn;
}

// Row in registers (NCH chunks of 8 bf16 per thread: a single HBM read), one fused block reduction
// of the per-thread (max, Σexp) pairs, LSE, and dlogits = (softmax − onehot)/n_valid in the same pass.
template <int NCH>
__global__ __launch_bounds__(XE_THREADS) void xent_kernel(const __bf16* __restrict__ logits, int ldl,
                                                          const int64_t* __restrict__ labels,
                                                          const int* __restrict__ n_valid, float* __restrict__ row_loss,
                                                          __bf16* __restrict__ dlogits, int S, int V) {
    __shared__ float red_m[XE_THREADS / 64], red_s[XE_THREADS / 64];
    __shared__ float tgt_logit;
    const int t = blockIdx.x;
    const int b = t / S, s = t % S;
    long long target = -100;
    if (s < S - 1) target = labels[(size_t)b * S + s + 1];
    const bool valid = target >= 0 && target < V;
    const __bf16* row = logits + (size_t)t * ldl;
    if (!valid) {
        if (threadIdx.x == 0) row_loss[t] = 0.f;
        if (dlogits) {
            bf16x8 z;
#pragma unroll
            for (int j = 0; j < 8; ++j) z[j] = f2bf(0.f);
            for (int ch = threadIdx.x; ch * 8 < ldl; ch += XE_THREADS)
                *reinterpret_cast<bf16x8*>(dlogits + (size_t)t * ldl + ch * 8) = z;
        }
        return;
    }
    bf16x8 x[NCH];
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
        const int ch = threadIdx.x + i * XE_THREADS;
        if (ch * 8 < ldl) x[i] = *reinterpret_cast<const bf16x8*>(row + ch * 8);
    }
    float mx = -INFINITY;
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
        const int ch = threadIdx.x + i * XE_THREADS;
        if (ch * 8 < ldl) {
#pragma unroll
            for (int j = 0; j < 8; ++j)
                if (ch * 8 + j < V) mx = fmaxf(mx, bf2f(x[i][j]));
        }
    }
    float se = 0.f;
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
        const int ch = threadIdx.x + i * XE_THREADS;
        if (ch * 8 < ldl) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int c = ch * 8 + j;
                if (c < V) se += __expf(bf2f(x[i][j]) - mx);
                if (c == target) tgt_logit = bf2f(x[i][j]);
            }
        }
    }
    // wave then block combine of (max, Σexp)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const float m2 = __shfl_xor(mx, o, 64), s2 = __shfl_xor(se, o, 64);
        ms_combine(mx, se, m2, s2);
    }
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (lane == 0) {
        red_m[wave] = mx;
        red_s[wave] = se;
    }
    __syncthreads();  // also publishes tgt_logit
    mx = red_m[0];
    se = red_s[0];
#pragma unroll
    for (int w = 1; w < XE_THREADS / 64; ++w) ms_combine(mx, se, red_m[w], red_s[w]);
    const float lse = mx + logf(se);
    if (threadIdx.x == 0) row_loss[t] = lse - tgt_logit;
    if (!dlogits) return;
    const float inv_n = 1.0f / (float)max(1, *n_valid);
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
        const int ch = threadIdx.x + i * XE_THREADS;
        if (ch * 8 < ldl) {
            bf16x8 d;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int c = ch * 8 + j;
                float g = 0.f;
                if (c < V) g = (__expf(bf2f(x[i][j]) - lse) - (c == target ? 1.f : 0.f)) * inv_n;
                d[j] = f2bf(g);
            }
            *reinterpret_cast<bf16x8*>(dlogits + (size_t)t * ldl + ch * 8) = d;
        }
    }
}

// counts[0] = LM rows the CE scores (label at s >= 1 scores logits row s-1; valid iff 0 <= y < V, the
// predicate xent_kernel uses), counts[1] = valid emotion labels (0 <= y < C; -100 = ignore_index).
__global__ __launch_bounds__(256) void count_valid_kernel(const int64_t* __restrict__ labels,
                                                          const int64_t* __restrict__ emo, int B, int S, int V, int C,
                                                          int* __restrict__ out) {
    __shared__ int red[2][4];
    int c = 0, ce = 0;
    if (labels)
        for (int i = threadIdx.x; i < B * S; i += 256) {
            const int64_t y = labels[i];
            if (i % S >= 1 && y >= 0 && y < V) ++c;
        }
    if (emo)
        for (int i = threadIdx.x; i < B; i += 256) ce += emo[i] >= 0 && emo[i] < C;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        c += __shfl_xor(c, o, 64);
        ce += __shfl_xor(ce, o, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        red[0][threadIdx.x >> 6] = c;
        red[1][threadIdx.x >> 6] = ce;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        out[0] = red[0][0] + red[0][1] + red[0][2] + red[0][3];
        out[1] = red[1][0] + red[1][1] + red[1][2] + red[1][3];
    }
}

// Emotion head, one workgroup per sample b: logits[b][c] = h[b,S-1,:]·W[c,:]; with labels the row
// loss and dlogits go to `scratch` ([B][C] dlogits then [B] row losses) and, with dh,
// dh[b,S-1,:] += dlogits[b]·W.  CrossEntropyLoss semantics (src/model.py:710-711): labels outside
// [0, C) (-100 = ignore_index) contribute neither loss nor gradient; the mean is over the n_valid
// (global) valid labels.
// Latency-bound (B workgroups, a few KB each): every global load of a phase is issued before the first use, so
// the phase pays one memory latency instead of one per loop iteration; the sums keep the lane-strided order.
constexpr int EMO_EV = 16;  // E <= 64 * EMO_EV (the LayerNorm kernels' limit, 1024)
__global__ __launch_bounds__(256) void emotion_row_kernel(const __bf16* __restrict__ h, const float* __restrict__ W,
                                                          const int64_t* __restrict__ labels, float* __restrict__ logits,
                                                          float* __restrict__ scratch, float* __restrict__ dh, int B, int S,
                                                          int E, int C, const int* __restrict__ n_valid,
                                                          const float* __restrict__ gscale) {
    __shared__ float lg[16], dl[16];
    const int b = blockIdx.x;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const __bf16* hr = h + ((size_t)b * S + S - 1) * E;
    float hv[EMO_EV];
#pragma unroll
    for (int k = 0; k < EMO_EV; ++k) hv[k] = lane + 64 * k < E ? bf2f(hr[lane + 64 * k]) : 0.f;
    for (int c = wave; c < C; c += 4) {
        const float* wr = W + (size_t)c * E;
        float wv[EMO_EV];
#pragma unroll
        for (int k = 0; k < EMO_EV; ++k) wv[k] = lane + 64 * k < E ? wr[lane + 64 * k] : 0.f;
        float acc = 0.f;
#pragma unroll
        for (int k = 0; k < EMO_EV; ++k)
            if (lane + 64 * k < E) acc += hv[k] * wv[k];
        acc = wave_sum(acc);
        if (lane == 0) {
            lg[c] = acc;
            logits[(size_t)b * C + c] = acc;
        }
    }
    __syncthreads();
    if (!labels) return;
    if (threadIdx.x == 0) {
        const float gs = gscale ? *gscale : 1.f;
        float mx = -INFINITY;
        for (int c = 0; c < C; ++c) mx = fmaxf(mx, lg[c]);
        float se = 0.f;
        for (int c = 0; c < C; ++c) se += expf(lg[c] - mx);
        const int64_t y = labels[b];
        const bool valid = y >= 0 && y < C;
        const float inv_n = 1.0f / (float)max(1, *n_valid);
        for (int c = 0; c < C; ++c) {
            const float d = valid ? (expf(lg[c] - mx) / se - (c == y ? 1.f : 0.f)) * gs * inv_n : 0.f;
            dl[c] = d;
            scratch[(size_t)b * C + c] = d;
        }
        scratch[(size_t)B * C + b] = valid ? (mx + logf(se)) - lg[y] : 0.f;
    }
    __syncthreads();
    if (!dh) return;
    float* dr = dh + ((size_t)b * S + S - 1) * E;
    constexpr int EPT = EMO_EV / 4;  // columns per thread (256 threads)
    float wv[EPT][16], o[EPT];
#pragma unroll
    for (int k = 0; k < EPT; ++k) {
        const int e = threadIdx.x + 256 * k;
        o[k] = e < E ? dr[e] : 0.f;
#pragma unroll
        for (int c = 0; c < 16; ++c) wv[k][c] = (c < C && e < E) ? W[(size_t)c * E + e] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < EPT; ++k) {
        const int e = threadIdx.x + 256 * k;
        if (e >= E) continue;
        float acc = 0.f;
#pragma unroll
        for (int c = 0; c < 16; ++c)
            if (c < C) acc += dl[c] * wv[k][c];
        dr[e] = o[k] + acc;
    }
}

// dW[c][e] = Σ_b dlogits[b][c]·h[b,S-1,e] (fixed b order); block 0 also sums the row losses.  The dlogits are
// staged in LDS and the h column of 16 samples is loaded at once, so a chunk pays one memory latency.
__global__ __launch_bounds__(256) void emotion_dw_kernel(const __bf16* __restrict__ h, const float* __restrict__ scratch,
                                                         float* __restrict__ loss_sum, float* __restrict__ dW, int B,
                                                         int S, int E, int C) {
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        float s = 0.f;
        for (int b = 0; b < B; ++b) s += scratch[(size_t)B * C + b];
        *loss_sum = s;
    }
    if (!dW) return;
    __shared__ float dl[16][16];
    const int e = blockIdx.x * 256 + threadIdx.x;
    float acc[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) acc[c] = 0.f;
    for (int b0 = 0; b0 < B; b0 += 16) {
        __syncthreads();
        {
            const int bb = threadIdx.x >> 4, c = threadIdx.x & 15;
            dl[bb][c] = (b0 + bb < B && c < C) ? scratch[(size_t)(b0 + bb) * C + c] : 0.f;
        }
        float hv[16];
#pragma unroll
        for (int j = 0; j < 16; ++j)
            hv[j] = (e < E && b0 + j < B) ? bf2f(h[((size_t)(b0 + j) * S + S - 1) * E + e]) : 0.f;
        __syncthreads();
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            if (b0 + j >= B) break;
#pragma unroll
            for (int c = 0; c < 16; ++c)
                if (c < C) acc[c] += dl[j][c] * hv[j];
        }
    }
    if (e >= E) return;
#pragma unroll
    for (int c = 0; c < 16; ++c)
        if (c < C) dW[(size_t)c * E + e] = acc[c];
}

// The trainer's running metrics (src/main.py:158-169: loss.item() sums and emotion argmax accuracy),
// accumulated on the device by the loss finalisation instead of a string of small framework kernels.
struct MetricAcc {
    float* loss_acc;             // [0] += total loss, [1] += LM loss (nullptr: off)
    unsigned long long* correct;  // += #(argmax(emo_logits[b]) == emo_labels[b])
    const float* emo_logits;     // [B][C]
    const int64_t* emo_labels;   // [B]
    int B, C;
};

__global__ __launch_bounds__(256) void loss_finalize_kernel(const float* __restrict__ row_loss, int T,
                                                            const int* __restrict__ n_valid,
                                                            const float* __restrict__ emo_sum,
                                                            const int* __restrict__ n_emo, float* __restrict__ out,
                                                            MetricAcc acc) {
    __shared__ float red[4];
    __shared__ int hits[4];
    float s = 0.f;
    for (int i = threadIdx.x; i < T; i += 256) s += row_loss[i];
    s = wave_sum(s);
    int h = 0;
    if (acc.correct && acc.emo_logits && acc.emo_labels) {
        for (int b = threadIdx.x; b < acc.B; b += 256) {  // torch argmax: the first index of the maximum
            const float* r = acc.emo_logits + (size_t)b * acc.C;
            int best = 0;
            for (int c = 1; c < acc.C; ++c)
                if (r[c] > r[best]) best = c;
            h += (int64_t)best == acc.emo_labels[b];
        }
    }
    h = (int)wave_sum((float)h);
    if ((threadIdx.x & 63) == 0) {
        red[threadIdx.x >> 6] = s;
        hits[threadIdx.x >> 6] = h;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        float lm = ((red[0] + red[1]) + red[2]) + red[3];
        // mean over the valid labels; none valid gives 0/0 = NaN, as torch's CrossEntropyLoss does for the
        // reference (src/model.py:704-709; the dlogits of ignored rows stay 0, as its gradient does)
        lm = n_valid ? lm / (float)(*n_valid) : 0.f;
        float emo = emo_sum ? *emo_sum / (float)(*n_emo) : 0.f;  // likewise 0/0 = NaN with no valid label
        out[0] = lm;
        out[1] = emo;
        out[2] = lm + emo;
        if (acc.loss_acc) {
            acc.loss_acc[0] += lm + emo;
            acc.loss_acc[1] += lm;
        }
        if (acc.correct) *acc.correct += (unsigned long long)(hits[0] + hits[1] + hits[2] + hits[3]);
    }
}

}  // namespace ergm

using namespace ergm;

extern "C" int ergm_count_valid(const int64_t* labels, const int64_t* emotion_labels, int B, int S, int V, int C,
                                int* counts, void* stream) {
    ERGM_CHECK_ARG(counts && B > 0 && S > 0 && V > 0 && C > 0, "count_valid: bad argument");
    ERGM_LAUNCH(count_valid_kernel, dim3(1), dim3(256), 0, as_stream(stream), labels, emotion_labels, B, S, V, C,
                       counts);
    return check_launch("count_valid");
}

extern "C" int ergm_xent_fwd_bwd(const void* logits, int ldl, const int64_t* labels, const int* n_valid_global,
                                 float* row_loss, void* dlogits, int B, int S, int V, float grad_scale, void* stream) {
    ERGM_CHECK_ARG(logits && labels && n_valid_global && row_loss, "xent: null argument");
    ERGM_CHECK_ARG(B > 0 && S > 0 && V > 0 && ldl >= V && ldl % 8 == 0, "xent: bad shape (ldl %% 8 == 0 required)");
    int nch = cdiv(cdiv(ldl, 8), XE_THREADS);
    ERGM_CHECK_ARG(nch <= XE_MAXCH, "xent: row of %d columns too long", ldl);
    ERGM_CHECK_ARG(grad_scale == 1.0f, "xent: grad_scale is applied by the consumer GEMMs (pass 1)");
    const auto* lg = reinterpret_cast<const __bf16*>(logits);
    auto* dl = reinterpret_cast<__bf16*>(dlogits);
    hipStream_t s = as_stream(stream);
    dim3 grid(B * S), blk(XE_THREADS);
    if (nch <= 2) ERGM_LAUNCH(xent_kernel<2>, grid, blk, 0, s, lg, ldl, labels, n_valid_global, row_loss, dl, S, V);
    else if (nch <= 4) ERGM_LAUNCH(xent_kernel<4>, grid, blk, 0, s, lg, ldl, labels, n_valid_global, row_loss, dl, S, V);
    else if (nch <= 8) ERGM_LAUNCH(xent_kernel<8>, grid, blk, 0, s, lg, ldl, labels, n_valid_global, row_loss, dl, S, V);
    else if (nch <= 13) ERGM_LAUNCH(xent_kernel<13>, grid, blk, 0, s, lg, ldl, labels, n_valid_global, row_loss, dl, S, V);
    else ERGM_LAUNCH(xent_kernel<16>, grid, blk, 0, s, lg, ldl, labels, n_valid_global, row_loss, dl, S, V);
    return check_launch("xent");
}

extern "C" int ergm_emotion_head(const void* h, const float* W, const int64_t* labels, float* logits, float* loss_sum,
                                 float* dW, float* dh, float* scratch, int B, int S, int E, int C,
                                 const int* n_valid_global, const float* grad_scale_dev, void* stream) {
    ERGM_CHECK_ARG(h && W && logits, "emotion_head: null argument");
    ERGM_CHECK_ARG(B > 0 && C > 0 && C <= 16 && E > 0 && E <= 64 * EMO_EV && S > 0, "emotion_head: bad shape");
    ERGM_CHECK_ARG(!labels || (loss_sum && scratch && n_valid_global), "emotion_head: labels need loss_sum, scratch and n_valid");
    ERGM_CHECK_ARG((dW == nullptr) == (dh == nullptr), "emotion_head: dW and dh go together");
    ERGM_CHECK_ARG(!dW || labels, "emotion_head: gradients need labels");
    hipStream_t s = as_stream(stream);
    const __bf16* hb = reinterpret_cast<const __bf16*>(h);
    ERGM_LAUNCH(emotion_row_kernel, dim3(B), dim3(256), 0, s, hb, W, labels, logits, scratch, dh, B, S, E, C,
                       n_valid_global, grad_scale_dev);
    if (labels)
        ERGM_LAUNCH(emotion_dw_kernel, dim3(dW ? cdiv(E, 256) : 1), dim3(256), 0, s, hb, scratch, loss_sum, dW,
                           B, S, E, C);
    return check_launch("emotion_head");
}

extern "C" int ergm_loss_finalize(const float* row_loss, int T, const int* n_valid_global, const float* emo_loss_sum,
                                  const int* n_valid_emo, float* out, void* stream) {
    ERGM_CHECK_ARG(row_loss && out && T > 0, "loss_finalize: bad argument");
    ERGM_CHECK_ARG(!emo_loss_sum || n_valid_emo, "loss_finalize: the emotion loss needs its valid count");
    ERGM_LAUNCH(loss_finalize_kernel, dim3(1), dim3(256), 0, as_stream(stream), row_loss, T, n_valid_global,
                       emo_loss_sum, n_valid_emo, out, MetricAcc{});
    return check_launch("loss_finalize");
}

namespace ergm {
// dl[i] = bf16(scale · dl[i] + g[i]) over n bf16 elements (8 per thread): a caller's gradient on the returned
// logits added to the cross-entropy's, both scaled as the LM-head backward GEMMs expect (alpha 1).
__global__ __launch_bounds__(256) void dlogits_add_kernel(bf16x8* __restrict__ dl, const bf16x8* __restrict__ g,
                                                          const float* __restrict__ scale, size_t n8) {
    const float sc = scale ? *scale : 1.0f;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (size_t)gridDim.x * blockDim.x) {
        bf16x8 a = dl[i];
        const bf16x8 b = g[i];
#pragma unroll
        for (int j = 0; j < 8; ++j) a[j] = f2bf(sc * bf2f(a[j]) + bf2f(b[j]));
        dl[i] = a;
    }
}
int dlogits_add(void* dl, const void* g, const float* scale, size_t n, hipStream_t s) {
    ERGM_CHECK_ARG(dl && g && n % 8 == 0 && aligned16(dl) && aligned16(g), "dlogits_add: bad argument");
    const size_t n8 = n / 8;
    const unsigned grid = (unsigned)std::min<size_t>((n8 + 255) / 256, 4096);
    ERGM_LAUNCH(dlogits_add_kernel, dim3(grid), dim3(256), 0, s, reinterpret_cast<bf16x8*>(dl),
                       reinterpret_cast<const bf16x8*>(g), scale, n8);
    return check_launch("dlogits_add");
}

// ergm_loss_finalize that also accumulates the trainer metrics (ergm_model_set_metrics).
int loss_finalize_metrics(const float* row_loss, int T, const int* n_valid_global, const float* emo_loss_sum,
                          const int* n_valid_emo, float* out, float* loss_acc, int64_t* correct,
                          const float* emo_logits, const int64_t* emo_labels, int B, int C, hipStream_t s) {
    MetricAcc acc{loss_acc, reinterpret_cast<unsigned long long*>(correct), emo_logits, emo_labels, B, C};
    ERGM_LAUNCH(loss_finalize_kernel, dim3(1), dim3(256), 0, s, row_loss, T, n_valid_global, emo_loss_sum,
                       n_valid_emo, out, acc);
    return check_launch("loss_finalize");
}
}  // namespace ergm
