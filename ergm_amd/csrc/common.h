// Internal helpers shared by the gfx950 kernels of libergm_hip.so.
#pragma once

#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>
#include <string>

#include "../../include/ergm_hip.h"

namespace ergm {

// ---- error state (thread-local; ergm_last_error reads it) ----------------------------------
void set_error(const char* fmt, ...);
int fail(int code, const char* fmt, ...);
int check_launch(const char* what);

#define ERGM_CHECK_ARG(cond, ...)                                   \
    do {                                                            \
        if (!(cond)) return ::ergm::fail(ERGM_EINVAL, __VA_ARGS__); \
    } while (0)
#define ERGM_TRY(expr)                 \
    do {                               \
        int _rc = (expr);              \
        if (_rc != ERGM_OK) return _rc; \
    } while (0)

// ---- kernel launches, and fork points bound to them ------------------------------------------
// Every kernel of the library is launched through ERGM_LAUNCH.  A cross-stream fork point made with
// hipEventRecord puts a marker packet of its own on the producing stream, which the stream's next kernel
// waits behind (~5 us per fork in the training step's backward); the same event bound to the producing
// kernel's own dispatch (hipExtLaunchKernel's stop event) costs the stream nothing.  bind_arm(s, ev)
// binds `ev` to every following ERGM_LAUNCH on stream s (so it ends up on the last one) until
// bind_take(s) returns it; bind_take returns nullptr when nothing was launched on s since the arm or
// the binding was cleared (bind_clear) — the caller then records the event itself.
struct LaunchBind {
    hipStream_t s = nullptr;
    hipEvent_t armed = nullptr;  // bound to each ERGM_LAUNCH on s while set
    bool bound = false;          // the latest launch on s carries `armed`
};
extern thread_local LaunchBind g_bind;
inline void bind_arm(hipStream_t s, hipEvent_t ev) { g_bind = LaunchBind{s, ev, false}; }
inline hipEvent_t bind_take(hipStream_t s) {
    hipEvent_t e = (g_bind.armed && g_bind.bound && g_bind.s == s) ? g_bind.armed : nullptr;
    g_bind = LaunchBind{};
    return e;
}
inline void bind_clear() { g_bind = LaunchBind{}; }

#define ERGM_LAUNCH(K, G, B, SH, S, ...)                                                        \
    do {                                                                                        \
        hipStream_t s_ = (S);                                                                   \
        if (::ergm::g_bind.armed && s_ == ::ergm::g_bind.s) {                                   \
            hipExtLaunchKernelGGL(K, G, B, SH, s_, nullptr, ::ergm::g_bind.armed, 0, __VA_ARGS__); \
            ::ergm::g_bind.bound = true;                                                        \
        } else {                                                                                \
            hipLaunchKernelGGL(K, G, B, SH, s_, __VA_ARGS__);                                   \
        }                                                                                       \
    } while (0)

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }
inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }
inline int cdiv(int a, int b) { return (a + b - 1) / b; }


// ---- device types -----------------------------------------------------------------------
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef uint16_t bf16_t;  // storage type on the host side / in pointer arithmetic

#define LDS_PTR(T, p) ((__attribute__((address_space(3))) T*)(p))

__device__ __forceinline__ float bf2f(__bf16 x) { return (float)x; }
__device__ __forceinline__ __bf16 f2bf(float x) { return (__bf16)x; }  // RNE (v_cvt_pk_bf16_f32)

__device__ __forceinline__ float bits2f(uint16_t b) { return __uint_as_float(((uint32_t)b) << 16); }

// fp8 weight quantisation jobs (quant.hip), batched over the matrices of one block
struct WqJob {
    const void* W;        // [K][ldw] f32 or bf16 (Conv1D [in, out]), see w_bf16
    uint8_t* Wt;          // [N][ldt] e4m3 (transposed)
    float* scale;         // [N]
    unsigned* amax;       // [N] |w| bit patterns, zeroed by the caller
    int ldw, K, N, ldt;
    int blk_amax, blk_q;  // first block of this job in each grid (set by quant_weights_fp8)
    int w_bf16;           // W is the bf16 shadow (the executor) rather than the f32 master
};
struct WqJobs {
    WqJob j[8];
    int n;
};
// MX-fp8 weight quantisation jobs (quant.hip): W [K][ldw] bf16 -> Wt [N][ldt] e4m3 (transposed) with an e8m0
// scale per (column, 32-row block): sc [N][lds]; optionally also the row form Wr [K][ldr] e4m3 with a scale per
// (row, 32-column block): scr [K][ldsr] (the B operand of the data-gradient GEMM dX = dY·Wᵀ)
struct MxJob {
    const __bf16* W;
    uint8_t* Wt;
    uint8_t* sc;
    int ldw, K, N, ldt, lds;
    int blk;  // first block of this job in the grid (set by quant_weights_mx)
    uint8_t* Wr;
    uint8_t* scr;
    int ldr, ldsr;
};
struct MxJobs {
    MxJob j[8];
    int n;
};

// wave-level reductions over 64 lanes, all VALU (no ds_bpermute round trips): DPP quad_perm [1,0,3,2]
// and [2,3,0,1], row_half_mirror and row_mirror inside each 16-lane row, then the gfx950 row swaps
// v_permlane16_swap / v_permlane32_swap across rows.  Every step combines a lane's value with its
// partner's by a commutative op, so all 64 lanes end with the bit-identical result.  Full waves only.
template <int CTRL>
__device__ __forceinline__ float dpp_f32(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
template <bool MAX>
__device__ __forceinline__ float wave_reduce(float v) {
    auto op = [](float a, float b) { return MAX ? fmaxf(a, b) : a + b; };
    v = op(v, dpp_f32<0xB1>(v));   // quad_perm [1,0,3,2]
    v = op(v, dpp_f32<0x4E>(v));   // quad_perm [2,3,0,1]
    v = op(v, dpp_f32<0x141>(v));  // row_half_mirror
    v = op(v, dpp_f32<0x140>(v));  // row_mirror
    auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = op(__uint_as_float(r[0]), __uint_as_float(r[1]));
    r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return op(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float wave_sum(float v) { return wave_reduce<false>(v); }
__device__ __forceinline__ float wave_max(float v) { return wave_reduce<true>(v); }

// gelu_new (transformers NewGELUActivation): 0.5x(1+tanh(sqrt(2/pi)(x+0.044715x^3)))
__device__ __forceinline__ float gelu_new(float x) {
    const float k0 = 0.7978845608028654f;  // sqrt(2/pi)
    float u = k0 * (x + 0.044715f * x * x * x);
    return 0.5f * x * (1.0f + tanhf(u));
}
// gelu_new(x) and its derivative from one tanh: the forward keeps the derivative for the backward
// (the GELU backward is then a plain product, no transcendental on the backward critical path)
__device__ __forceinline__ float gelu_new_fwd(float x, float& dgelu) {
    const float k0 = 0.7978845608028654f;
    const float x2 = x * x;
    const float t = tanhf(k0 * (x + 0.044715f * x2 * x));
    dgelu = 0.5f * (1.0f + t) + 0.5f * x * (1.0f - t * t) * k0 * (1.0f + 3.0f * 0.044715f * x2);
    return 0.5f * x * (1.0f + t);
}
__device__ __forceinline__ float gelu_new_grad(float x) {
    const float k0 = 0.7978845608028654f;
    float x2 = x * x;
    float u = k0 * (x + 0.044715f * x2 * x);
    float t = tanhf(u);
    return 0.5f * (1.0f + t) + 0.5f * x * (1.0f - t * t) * k0 * (1.0f + 3.0f * 0.044715f * x2);
}

// ---- torch.optim.AdamW (src/main.py:68,155), single-tensor algorithm in torch's arithmetic order ----------------
//   p *= 1 - lr·wd;  m = m + (1-β1)(g - m)  (lerp);  v = β2·v + (1-β2)·g·g  (addcmul)
//   p += -step_size · m / (sqrt(v)/bc2_sqrt + eps)           (addcdiv)
// One element.  No FMA contraction: the optimizer passes of adamw.hip (whole ranges and selected wte rows) must round
// identically.
struct AdamScalars {
    float decay, one_m_b1, b2, one_m_b2, eps, step_size, bc2_sqrt;
};
__device__ __forceinline__ float adamw_elem(float p, float g, float& m, float& v, const AdamScalars& s) {
#pragma clang fp contract(off)
    float x = p * s.decay;
    const float mj = m + s.one_m_b1 * (g - m);
    const float vj = v * s.b2 + s.one_m_b2 * (g * g);
    const float denom = sqrtf(vj) / s.bc2_sqrt + s.eps;
    x = x + (-s.step_size) * (mj / denom);
    m = mj;
    v = vj;
    return x;
}
// The scalar products torch forms in double and rounds once when applied to fp32 tensors.
AdamScalars adam_scalars(double lr, double beta1, double beta2, float eps, double weight_decay, float step_size,
                         float bc2_sqrt);

__device__ __forceinline__ f32x4 ld_nt4(const float* p) {
    return __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p));
}
__device__ __forceinline__ void st_nt4(float* p, f32x4 x) { __builtin_nontemporal_store(x, reinterpret_cast<f32x4*>(p)); }

// ---- dropout (nn.Dropout at src/model.py:142,245,266,506) -------------------------------------
// Counter-based: the keep decision of element (row, col) of dropout site `site` in forward number
// `offset` is a pure function of (seed, offset, site, global row, col), so the backward recomputes
// it instead of storing it.  Random words: Philox4x32-10 (Salmon et al., SC'11; Random123), one call
// per group of 4 consecutive columns: counter = {g_lo, g_hi, site, offset} with
// g = row·ceil(cols/4) + col/4, key = seed; element col uses word col & 3.  Dropped iff word < thresh
// (thresh = round(p·2^32)); kept elements are scaled by 1/(1-p) as torch's dropout does.
struct DropSite {
    uint32_t key0, key1;  // seed
    uint32_t site;        // counter word 2: which nn.Dropout (ergm_hip.h ERGM_DROP_SITE_*)
    uint32_t offset;      // counter word 3: forward number
    uint32_t thresh;      // 0: dropout off
    float scale;          // 1 / (1 - p)
    int64_t row0;         // global row of the caller's row 0 (DP ranks / batch-half chains)
    int64_t cols4;        // ceil(cols / 4): counter groups per row
};

__device__ __forceinline__ uint4 philox4x32_10(uint4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c.x, p1 = (uint64_t)0xCD9E8D57u * c.z;
        c = make_uint4((uint32_t)(p1 >> 32) ^ c.y ^ k0, (uint32_t)p1, (uint32_t)(p0 >> 32) ^ c.w ^ k1, (uint32_t)p0);
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return c;
}

// Keep bits of columns col..col+3 (col % 4 == 0) of `row` (caller-relative): bit j = column col+j kept.
__device__ __forceinline__ unsigned drop_keep4(const DropSite& d, int64_t row, int col) {
    const uint64_t g = (uint64_t)(d.row0 + row) * (uint64_t)d.cols4 + (uint64_t)(col >> 2);
    const uint4 r = philox4x32_10(make_uint4((uint32_t)g, (uint32_t)(g >> 32), d.site, d.offset), d.key0, d.key1);
    return (r.x >= d.thresh ? 1u : 0u) | (r.y >= d.thresh ? 2u : 0u) | (r.z >= d.thresh ? 4u : 0u) |
           (r.w >= d.thresh ? 8u : 0u);
}
// Single element (any col): the word col & 3 of its group.
__device__ __forceinline__ bool drop_keep1(const DropSite& d, int64_t row, int col) {
    return (drop_keep4(d, row, col & ~3) >> (col & 3)) & 1u;
}

// ---- MX-fp8 (OCP microscaling) helpers: 32-element blocks, e8m0 block scale 2^(e-127), e4m3fn elements ----
// Block exponent: the smallest e with amax <= 448·2^e (no element saturates), from the bits of amax: amax =
// 1.f·2^ea gives e = ea - 8, or ea - 7 when 1.f > 1.75 (448 = 1.75·2^8).  A zero block gets e = 0 (scale 1).
// Returned biased (e + 127, clamped to [0, 254]); the scaled values v·2^-e are exact in f32.
// MX scale layout: the e8m0 bytes of a 128-deep K step (4 blocks) of every row are one 4-byte word, and the words of
// one K step are contiguous over the rows: byte (row, block b) at ((b / 4) * pitch + row) * 4 + b % 4, pitch >= the
// row count.  A GEMM stage's scale loads are then whole cache lines (64 rows = 256 contiguous bytes) instead of one
// 4-byte piece of 64 different rows.
__device__ __forceinline__ size_t mx_sidx(int row, int blk, int pitch) {
    return ((size_t)(blk >> 2) * pitch + row) * 4 + (blk & 3);
}
__device__ __forceinline__ int mx_exp_biased(float amax) {
    const uint32_t b = __float_as_uint(amax);
    if (amax == 0.f) return 127;
    const int ea = (int)((b >> 23) & 0xff) - 127;
    const int e = ea - 8 + ((b & 0x7fffff) > 0x600000u ? 1 : 0);
    return min(max(e + 127, 0), 254);
}
__device__ __forceinline__ float mx_inv_scale(int eb) { return __uint_as_float((uint32_t)(254 - eb) << 23); }  // 2^-(eb-127)
__device__ __forceinline__ uint32_t mx_pack4(float a, float b, float c, float d) {
    a = fminf(fmaxf(a, -448.f), 448.f);
    b = fminf(fmaxf(b, -448.f), 448.f);
    c = fminf(fmaxf(c, -448.f), 448.f);
    d = fminf(fmaxf(d, -448.f), 448.f);
    int q = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
    q = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, q, true);
    return (uint32_t)q;
}
// 8 consecutive values of a 32-element block held by 4 consecutive lanes (lane & 3 = position in the block):
// block amax across the 4 lanes, then 8 e4m3 bytes; returns the biased block exponent
__device__ __forceinline__ int mx_quant8_x4(const float* v, uint2& q) {
    float am = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) am = fmaxf(am, fabsf(v[j]));
    am = fmaxf(am, __shfl_xor(am, 1, 64));
    am = fmaxf(am, __shfl_xor(am, 2, 64));
    const int eb = mx_exp_biased(am);
    const float is = mx_inv_scale(eb);
    q.x = mx_pack4(v[0] * is, v[1] * is, v[2] * is, v[3] * is);
    q.y = mx_pack4(v[4] * is, v[5] * is, v[6] * is, v[7] * is);
    return eb;
}

// Host: the descriptor of one site (p in [0, 1); p == 0 gives thresh 0 = off).
DropSite make_drop_site(uint64_t seed, uint32_t offset, uint32_t site, float p, int64_t row0, int64_t cols);
DropSite drop_site_of(const ergm_dropout* d, int64_t cols);  // NULL or p == 0: off
int check_dropout(const ergm_dropout* d);
int dropout_apply_f32(const DropSite& d, float* x, int rows, int cols, int ld, hipStream_t s);

}  // namespace ergm
