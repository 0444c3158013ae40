// Cross-entropy losses of GPT2LMHeadModel for gfx950.
//
// LM loss: CrossEntropyLoss(ignore_index=-100, mean) on logits[..., :-1, :] vs labels[..., 1:]
// (src/model.py:704-708) — one workgroup per logits row keeps the whole bf16 row in registers
// (single HBM read), computes max / Σexp / LSE with wave shuffles, and writes
// dlogits = (softmax − onehot)/n_valid in the same pass (forward and backward fused; the shift is
// pure indexing: row (b, s) is scored against labels[b][s+1]).
// Emotion loss: emotion_head on the last token + CrossEntropyLoss (src/model.py:700-701,710-711).
#include "common.h"

namespace ergm {

constexpr int XE_THREADS = 256;
constexpr int XE_MAXCH = 32;  // 16-B chunks per thread: rows up to 32*256*8 = 65536 columns

__device__ __forceinline__ float block_reduce(float v, float* red, bool is_max) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    v = is_max ? wave_max(v) : wave_sum(v);
    __syncthreads();
    if (lane == 0) red[wave] = v;
    __syncthreads();
    float r = red[0];
#pragma unroll
    for (int w = 1; w < XE_THREADS / 64; ++w) r = is_max ? fmaxf(r, red[w]) : r + red[w];
    return r;
}

__global__ __launch_bounds__(XE_THREADS) void xent_kernel(const __bf16* __restrict__ logits, int ldl,
                                                          const int64_t* __restrict__ labels,
                                                          const int* __restrict__ n_valid, float* __restrict__ row_loss,
                                                          __bf16* __restrict__ dlogits, int S, int V, int nch) {
    __shared__ float red[XE_THREADS / 64];
    __shared__ float tgt_logit;
    const int t = blockIdx.x;
    const int b = t / S, s = t % S;
    long long target = -100;
    if (s < S - 1) target = labels[(size_t)b * S + s + 1];
    const bool valid = target >= 0 && target < V;
    const __bf16* row = logits + (size_t)t * ldl;
    bf16x8 x[XE_MAXCH];
    float mx = -INFINITY;
#pragma unroll
    for (int i = 0; i < XE_MAXCH; ++i) {
        int ch = threadIdx.x + i * XE_THREADS;
        if (i < nch && ch * 8 < ldl) {
            x[i] = *reinterpret_cast<const bf16x8*>(row + ch * 8);
#pragma unroll
            for (int j = 0; j < 8; ++j)
                if (ch * 8 + j < V) mx = fmaxf(mx, bf2f(x[i][j]));
        }
    }
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
    mx = block_reduce(mx, red, true);
    float se = 0.f;
#pragma unroll
    for (int i = 0; i < XE_MAXCH; ++i) {
        int ch = threadIdx.x + i * XE_THREADS;
        if (i < nch && ch * 8 < ldl) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                int c = ch * 8 + j;
                if (c < V) se += __expf(bf2f(x[i][j]) - mx);
                if (c == target) tgt_logit = bf2f(x[i][j]);
            }
        }
    }
    se = block_reduce(se, red, false);  // its barriers also publish tgt_logit
    const float lse = mx + logf(se);
    if (threadIdx.x == 0) row_loss[t] = lse - tgt_logit;
    if (!dlogits) return;
    const float inv_n = 1.0f / (float)max(1, *n_valid);
    const float inv_se = 1.0f / se;
#pragma unroll
    for (int i = 0; i < XE_MAXCH; ++i) {
        int ch = threadIdx.x + i * XE_THREADS;
        if (i < nch && ch * 8 < ldl) {
            bf16x8 d;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                int c = ch * 8 + j;
                float g = 0.f;
                if (c < V) g = (__expf(bf2f(x[i][j]) - mx) * inv_se - (c == target ? 1.f : 0.f)) * inv_n;
                d[j] = f2bf(g);
            }
            *reinterpret_cast<bf16x8*>(dlogits + (size_t)t * ldl + ch * 8) = d;
        }
    }
}

__global__ __launch_bounds__(256) void count_valid_kernel(const int64_t* __restrict__ labels, int B, int S,
                                                          int* __restrict__ out) {
    __shared__ int red[4];
    int c = 0;
    for (int i = threadIdx.x; i < B * S; i += 256) {
        int s = i % S;
        if (s >= 1 && labels[i] != -100) ++c;  // label at s scores logits row s-1
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) *out = red[0] + red[1] + red[2] + red[3];
}

// Single workgroup: emotion logits (f32) + CE + gradients.  C ≤ 16, B ≤ 256.
__global__ __launch_bounds__(256) void emotion_kernel(const __bf16* __restrict__ h, const float* __restrict__ W,
                                                      const int64_t* __restrict__ labels, float* __restrict__ logits,
                                                      float* __restrict__ loss_sum, float* __restrict__ dW,
                                                      float* __restrict__ dh, int B, int S, int E, int C, int B_global,
                                                      const float* __restrict__ gscale) {
    extern __shared__ float sm[];
    float* lg = sm;            // [B][C] logits
    float* dl = sm + B * C;    // [B][C] dlogits
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int pc = wave; pc < B * C; pc += 4) {
        int b = pc / C, c = pc % C;
        const __bf16* hr = h + ((size_t)b * S + S - 1) * E;
        const float* wr = W + (size_t)c * E;
        float acc = 0.f;
        for (int e = lane; e < E; e += 64) acc += bf2f(hr[e]) * wr[e];
        acc = wave_sum(acc);
        if (lane == 0) {
            lg[pc] = acc;
            logits[pc] = acc;
        }
    }
    __syncthreads();
    if (!labels) return;
    const float gs = gscale ? *gscale : 1.f;
    if (threadIdx.x < B) {
        int b = threadIdx.x;
        float mx = -INFINITY;
        for (int c = 0; c < C; ++c) mx = fmaxf(mx, lg[b * C + c]);
        float se = 0.f;
        for (int c = 0; c < C; ++c) se += expf(lg[b * C + c] - mx);
        int y = (int)labels[b];
        for (int c = 0; c < C; ++c)
            dl[b * C + c] = (expf(lg[b * C + c] - mx) / se - (c == y ? 1.f : 0.f)) * gs / (float)B_global;
        lg[b * C + 0] = (mx + logf(se)) - lg[b * C + y];  // reuse slot 0 for the row loss
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        float s = 0.f;
        for (int b = 0; b < B; ++b) s += lg[b * C];
        *loss_sum = s;
    }
    if (!dW) return;
    for (int i = threadIdx.x; i < C * E; i += 256) {
        int c = i / E, e = i % E;
        float acc = 0.f;
        for (int b = 0; b < B; ++b) acc += dl[b * C + c] * bf2f(h[((size_t)b * S + S - 1) * E + e]);
        dW[i] = acc;
    }
    for (int i = threadIdx.x; i < B * E; i += 256) {
        int b = i / E, e = i % E;
        float acc = 0.f;
        for (int c = 0; c < C; ++c) acc += dl[b * C + c] * W[(size_t)c * E + e];
        dh[((size_t)b * S + S - 1) * E + e] += acc;
    }
}

__global__ __launch_bounds__(256) void loss_finalize_kernel(const float* __restrict__ row_loss, int T,
                                                            const int* __restrict__ n_valid,
                                                            const float* __restrict__ emo_sum, int B_global,
                                                            float* __restrict__ out) {
    __shared__ float red[4];
    float s = 0.f;
    for (int i = threadIdx.x; i < T; i += 256) s += row_loss[i];
    s = wave_sum(s);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        float lm = ((red[0] + red[1]) + red[2]) + red[3];
        lm = n_valid ? lm / (float)max(1, *n_valid) : 0.f;
        float emo = emo_sum ? *emo_sum / (float)B_global : 0.f;
        out[0] = lm;
        out[1] = emo;
        out[2] = lm + emo;
    }
}

}  // namespace ergm

using namespace ergm;

extern "C" int ergm_count_valid(const int64_t* labels, int B, int S, int* n_valid, void* stream) {
    ERGM_CHECK_ARG(labels && n_valid && B > 0 && S > 0, "count_valid: bad argument");
    hipLaunchKernelGGL(count_valid_kernel, dim3(1), dim3(256), 0, as_stream(stream), labels, B, S, n_valid);
    return check_launch("count_valid");
}

extern "C" int ergm_xent_fwd_bwd(const void* logits, int ldl, const int64_t* labels, const int* n_valid_global,
                                 float* row_loss, void* dlogits, int B, int S, int V, float grad_scale, void* stream) {
    ERGM_CHECK_ARG(logits && labels && n_valid_global && row_loss, "xent: null argument");
    ERGM_CHECK_ARG(B > 0 && S > 0 && V > 0 && ldl >= V && ldl % 8 == 0, "xent: bad shape (ldl %% 8 == 0 required)");
    int nch = cdiv(cdiv(ldl, 8), XE_THREADS);
    ERGM_CHECK_ARG(nch <= XE_MAXCH, "xent: row of %d columns too long", ldl);
    ERGM_CHECK_ARG(grad_scale == 1.0f, "xent: grad_scale is applied by the consumer GEMMs (pass 1)");
    hipLaunchKernelGGL(xent_kernel, dim3(B * S), dim3(XE_THREADS), 0, as_stream(stream),
                       reinterpret_cast<const __bf16*>(logits), ldl, labels, n_valid_global, row_loss,
                       reinterpret_cast<__bf16*>(dlogits), S, V, nch);
    return check_launch("xent");
}

extern "C" int ergm_emotion_head(const void* h, const float* W, const int64_t* labels, float* logits, float* loss_sum,
                                 float* dW, float* dh, int B, int S, int E, int C, int B_global,
                                 const float* grad_scale_dev, void* stream) {
    ERGM_CHECK_ARG(h && W && logits, "emotion_head: null argument");
    ERGM_CHECK_ARG(B > 0 && B <= 256 && C > 0 && C <= 16 && E > 0 && S > 0, "emotion_head: bad shape");
    ERGM_CHECK_ARG(!labels || loss_sum, "emotion_head: labels need loss_sum");
    ERGM_CHECK_ARG((dW == nullptr) == (dh == nullptr), "emotion_head: dW and dh go together");
    ERGM_CHECK_ARG(!dW || labels, "emotion_head: gradients need labels");
    size_t lds = 2 * (size_t)B * C * sizeof(float);
    hipLaunchKernelGGL(emotion_kernel, dim3(1), dim3(256), lds, as_stream(stream), reinterpret_cast<const __bf16*>(h),
                       W, labels, logits, loss_sum, dW, dh, B, S, E, C, B_global > 0 ? B_global : B, grad_scale_dev);
    return check_launch("emotion_head");
}

extern "C" int ergm_loss_finalize(const float* row_loss, int T, const int* n_valid_global, const float* emo_loss_sum,
                                  int B_global, float* out, void* stream) {
    ERGM_CHECK_ARG(row_loss && out && T > 0, "loss_finalize: bad argument");
    hipLaunchKernelGGL(loss_finalize_kernel, dim3(1), dim3(256), 0, as_stream(stream), row_loss, T, n_valid_global,
                       emo_loss_sum, B_global > 0 ? B_global : 1, out);
    return check_launch("loss_finalize");
}
