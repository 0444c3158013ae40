// Fused AdamW over the flat fp32 parameter buffer for gfx950 (one launch for all 150M+ params).
//
// Replaces torch.optim.AdamW(model.parameters(), lr) .step() (src/main.py:68,155) — the
// single-tensor algorithm, in its arithmetic order:
//   p *= 1 - lr·wd;  m = m + (1-β1)(g - m)  (lerp);  v = β2·v + (1-β2)·g·g  (addcmul)
//   p += -step_size · m / (sqrt(v)/bc2_sqrt + eps)           (addcdiv)
// and refreshes the bf16 shadow copy the GEMMs read, in the same pass (HBM-bound: 30 B/param).
#include "common.h"

#include <algorithm>
#include <cstdlib>

namespace ergm {

__device__ __forceinline__ void adamw_one(float4& pp, const float4& gg, float4& mm, float4& vv, bf16x4& ob,
                                          const AdamScalars& s) {
    float* P = reinterpret_cast<float*>(&pp);
    const float* G = reinterpret_cast<const float*>(&gg);
    float* Mv = reinterpret_cast<float*>(&mm);
    float* Vv = reinterpret_cast<float*>(&vv);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        P[j] = adamw_elem(P[j], G[j], Mv[j], Vv[j], s);
        ob[j] = f2bf(P[j]);
    }
}

__device__ __forceinline__ float4 nt_load4(const float4* p) {  // gradients are read exactly once
    f32x4 t = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p));
    return make_float4(t[0], t[1], t[2], t[3]);
}

__device__ __forceinline__ void nt_store4(float4* p, const float4& x) {
    __builtin_nontemporal_store(f32x4{x.x, x.y, x.z, x.w}, reinterpret_cast<f32x4*>(p));
}
template <bool NT>
__device__ __forceinline__ float4 ld4(const float4* p) {
    if constexpr (NT) return nt_load4(p);
    else return *p;
}
template <bool NT>
__device__ __forceinline__ void st4(float4* p, const float4& x) {
    if constexpr (NT) nt_store4(p, x);
    else *p = x;
}

// Two float4 groups per thread per iteration (8 independent 16-B loads in flight before any math).
// NT: parameters and moments are also streamed with non-temporal loads / stores (each is touched once
// per step), so the pass does not evict the operands of the GEMMs it overlaps.
template <bool NT>
__global__ __launch_bounds__(256) void adamw_kernel(float4* __restrict__ p, const float4* __restrict__ g,
                                                    float4* __restrict__ m, float4* __restrict__ v,
                                                    bf16x4* __restrict__ pb, size_t n4, AdamScalars sc) {
    const size_t stride = (size_t)gridDim.x * 256;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += 2 * stride) {
        const size_t i2 = i + stride;
        const bool two = i2 < n4;
        float4 p0 = ld4<NT>(p + i), g0 = nt_load4(g + i), m0 = ld4<NT>(m + i), v0 = ld4<NT>(v + i);
        float4 p1, g1, m1, v1;
        if (two) {
            p1 = ld4<NT>(p + i2);
            g1 = nt_load4(g + i2);
            m1 = ld4<NT>(m + i2);
            v1 = ld4<NT>(v + i2);
        }
        bf16x4 o0, o1;
        adamw_one(p0, g0, m0, v0, o0, sc);
        st4<NT>(p + i, p0);
        st4<NT>(m + i, m0);
        st4<NT>(v + i, v0);
        if (pb) pb[i] = o0;
        if (two) {
            adamw_one(p1, g1, m1, v1, o1, sc);
            st4<NT>(p + i2, p1);
            st4<NT>(m + i2, m1);
            st4<NT>(v + i2, v1);
            if (pb) pb[i2] = o1;
        }
    }
}

__global__ __launch_bounds__(256) void cast_bf16_kernel(const float4* __restrict__ src, bf16x4* __restrict__ dst,
                                                        size_t n4) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) {
        float4 x = src[i];
        bf16x4 o;
        o[0] = f2bf(x.x); o[1] = f2bf(x.y); o[2] = f2bf(x.z); o[3] = f2bf(x.w);
        dst[i] = o;
    }
}

__global__ __launch_bounds__(256) void axpy_kernel(const float4* __restrict__ x, float4* __restrict__ y, size_t n4,
                                                   float alpha) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) {
        float4 a = x[i], b = y[i];
        b.x += alpha * a.x; b.y += alpha * a.y; b.z += alpha * a.z; b.w += alpha * a.w;
        y[i] = b;
    }
}

// Row-selective AdamW over a [rows][row_len] block: row r is updated iff (flag[r] != 0) == select.  Flat over the
// block's float4 groups like adamw_kernel (two per thread per iteration, non-temporal parameter / moment traffic, every
// lane busy); a group of a skipped row costs its row's flag byte (L1 / L2-resident: a row is 192 groups at E = 768).
// Round 4's one-workgroup-per-row form ran the 88 %-selected untouched-row pass at 4.9 TB/s (192 of 256 lanes, one
// group per thread, cached parameter traffic).
__global__ __launch_bounds__(256) void adamw_rows_kernel(float4* __restrict__ p, const float4* __restrict__ g,
                                                         float4* __restrict__ m, float4* __restrict__ v,
                                                         bf16x4* __restrict__ pb, size_t n4, int row4,
                                                         const uint8_t* __restrict__ flag, int select, AdamScalars sc) {
    const size_t stride = (size_t)gridDim.x * 256;
    const bool want = select != 0;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += 2 * stride) {
        const size_t i2 = i + stride;
        const bool on0 = (flag[(unsigned)i / (unsigned)row4] != 0) == want;  // n4 < 2^32 (host check)
        const bool on1 = i2 < n4 && (flag[(unsigned)i2 / (unsigned)row4] != 0) == want;
        float4 p0, g0, m0, v0, p1, g1, m1, v1;
        if (on0) { p0 = ld4<true>(p + i); g0 = nt_load4(g + i); m0 = ld4<true>(m + i); v0 = ld4<true>(v + i); }
        if (on1) { p1 = ld4<true>(p + i2); g1 = nt_load4(g + i2); m1 = ld4<true>(m + i2); v1 = ld4<true>(v + i2); }
        bf16x4 o0, o1;
        if (on0) {
            adamw_one(p0, g0, m0, v0, o0, sc);
            st4<true>(p + i, p0);
            st4<true>(m + i, m0);
            st4<true>(v + i, v0);
            if (pb) pb[i] = o0;
        }
        if (on1) {
            adamw_one(p1, g1, m1, v1, o1, sc);
            st4<true>(p + i2, p1);
            st4<true>(m + i2, m1);
            st4<true>(v + i2, v1);
            if (pb) pb[i2] = o1;
        }
    }
}

AdamScalars adam_scalars(double lr, double beta1, double beta2, float eps, double weight_decay, float step_size,
                         float bc2_sqrt) {
    // the scalar products torch forms in double and rounds once when applied to fp32 tensors
    return AdamScalars{(float)(1.0 - lr * weight_decay), (float)(1.0 - beta1), (float)beta2, (float)(1.0 - beta2), eps,
                       step_size, bc2_sqrt};
}

static unsigned grid_for(size_t n4) {
    size_t blocks = (n4 + 255) / 256;
    return (unsigned)(blocks < 8192 ? (blocks ? blocks : 1) : 8192);
}

static unsigned grid_for2(size_t n4) {  // adamw: each thread covers two strided float4 groups
    size_t blocks = (n4 + 511) / 512;
    return (unsigned)(blocks < 4096 ? (blocks ? blocks : 1) : 4096);
}

}  // namespace ergm

using namespace ergm;

extern "C" int ergm_adamw_step(float* p, const float* g, float* m, float* v, void* p_bf16, size_t n, double lr,
                               double beta1, double beta2, float eps, double weight_decay, float step_size,
                               float bc2_sqrt, int max_blocks, void* stream) {
    ERGM_CHECK_ARG(p && g && m && v, "adamw: null argument");
    ERGM_CHECK_ARG(max_blocks >= 0, "adamw: max_blocks must be >= 0");
    ERGM_CHECK_ARG(n % 4 == 0, "adamw: n must be a multiple of 4");
    ERGM_CHECK_ARG(aligned16(p) && aligned16(g) && aligned16(m) && aligned16(v), "adamw: 16-byte alignment");
    ERGM_CHECK_ARG(!p_bf16 || (reinterpret_cast<uintptr_t>(p_bf16) & 7) == 0, "adamw: bf16 copy alignment");
    size_t n4 = n / 4;
    if (n4 == 0) return ERGM_OK;
    const AdamScalars sc = adam_scalars(lr, beta1, beta2, eps, weight_decay, step_size, bc2_sqrt);
    unsigned grid = grid_for2(n4);
    if (max_blocks > 0 && grid > (unsigned)max_blocks) grid = (unsigned)max_blocks;
    // non-temporal parameter / moment traffic: C2 +1.2 %, C5 +0.6 % (profiles/r01_overlap_experiments.txt #15)
    ERGM_LAUNCH(adamw_kernel<true>, dim3(grid), dim3(256), 0, as_stream(stream), (float4*)p, (const float4*)g,
                (float4*)m, (float4*)v, (bf16x4*)p_bf16, n4, sc);
    return check_launch("adamw");
}

extern "C" int ergm_adamw_rows(float* p, const float* g, float* m, float* v, void* p_bf16, int rows, int row_len,
                               const void* row_flag, int select, double lr, double beta1, double beta2, float eps,
                               double weight_decay, float step_size, float bc2_sqrt, int max_blocks, void* stream) {
    ERGM_CHECK_ARG(p && g && m && v && row_flag, "adamw_rows: null argument");
    ERGM_CHECK_ARG(rows >= 0 && row_len > 0 && row_len % 4 == 0, "adamw_rows: row_len must be a positive multiple of 4");
    ERGM_CHECK_ARG(max_blocks >= 0, "adamw_rows: max_blocks must be >= 0");
    ERGM_CHECK_ARG(aligned16(p) && aligned16(g) && aligned16(m) && aligned16(v), "adamw_rows: 16-byte alignment");
    ERGM_CHECK_ARG(!p_bf16 || (reinterpret_cast<uintptr_t>(p_bf16) & 7) == 0, "adamw_rows: bf16 copy alignment");
    if (rows == 0) return ERGM_OK;
    const AdamScalars sc = adam_scalars(lr, beta1, beta2, eps, weight_decay, step_size, bc2_sqrt);
    const size_t n4 = (size_t)rows * (row_len / 4);
    ERGM_CHECK_ARG(n4 < ((size_t)1 << 32), "adamw_rows: block of %zu float4 groups too large", n4);
    unsigned grid = grid_for2(n4);
    if (max_blocks > 0 && grid > (unsigned)max_blocks) grid = (unsigned)max_blocks;
    ERGM_LAUNCH(adamw_rows_kernel, dim3(grid), dim3(256), 0, as_stream(stream), (float4*)p, (const float4*)g,
                       (float4*)m, (float4*)v, (bf16x4*)p_bf16, n4, row_len / 4, (const uint8_t*)row_flag, select,
                       sc);
    return check_launch("adamw_rows");
}

extern "C" int ergm_cast_bf16(const float* src, void* dst, size_t n, void* stream) {
    ERGM_CHECK_ARG(src && dst && n % 4 == 0, "cast_bf16: bad argument");
    size_t n4 = n / 4;
    if (n4 == 0) return ERGM_OK;
    ERGM_LAUNCH(cast_bf16_kernel, dim3(grid_for(n4)), dim3(256), 0, as_stream(stream), (const float4*)src,
                       (bf16x4*)dst, n4);
    return check_launch("cast_bf16");
}

extern "C" int ergm_axpy(const float* x, float* y, size_t n, float alpha, void* stream) {
    ERGM_CHECK_ARG(x && y && n % 4 == 0, "axpy: bad argument");
    size_t n4 = n / 4;
    if (n4 == 0) return ERGM_OK;
    ERGM_LAUNCH(axpy_kernel, dim3(grid_for(n4)), dim3(256), 0, as_stream(stream), (const float4*)x, (float4*)y,
                       n4, alpha);
    return check_launch("axpy");
}

// ---- data-parallel gradient exchange in bf16 with fp32 accumulation (ergm_amd/dist.py) ----------
// Each rank receives one chunk of every rank's bf16 gradient (all-to-all), sums the world copies of its
// chunk in fp32 in rank order (deterministic, the same sum whichever rank owns it), rounds once to
// bf16 and all-gathers: half the bytes of an fp32 all-reduce, one rounding of the reduced value.
namespace ergm {
__global__ __launch_bounds__(256) void chunk_sum_kernel(const bf16x4* __restrict__ in, int nchunks, size_t chunk4,
                                                        bf16x4* __restrict__ out) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < chunk4; i += (size_t)gridDim.x * 256) {
        float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int j = 0; j < nchunks; ++j) {
            const bf16x4 v = in[(size_t)j * chunk4 + i];
            s.x += bf2f(v[0]); s.y += bf2f(v[1]); s.z += bf2f(v[2]); s.w += bf2f(v[3]);
        }
        bf16x4 o;
        o[0] = f2bf(s.x); o[1] = f2bf(s.y); o[2] = f2bf(s.z); o[3] = f2bf(s.w);
        out[i] = o;
    }
}

// The same sum, rounded once to bf16 and written back widened to fp32 straight into the gradient (ZeRO-1:
// this rank's reduced chunk), for the first n4 groups only (the last rank's chunk may be short).
__global__ __launch_bounds__(256) void chunk_sum_f32_kernel(const bf16x4* __restrict__ in, int nchunks, size_t chunk4,
                                                            size_t n4, float4* __restrict__ out) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) {
        float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int j = 0; j < nchunks; ++j) {
            const bf16x4 v = in[(size_t)j * chunk4 + i];
            s.x += bf2f(v[0]); s.y += bf2f(v[1]); s.z += bf2f(v[2]); s.w += bf2f(v[3]);
        }
        out[i] = make_float4(bf2f(f2bf(s.x)), bf2f(f2bf(s.y)), bf2f(f2bf(s.z)), bf2f(f2bf(s.w)));
    }
}

// ZeRO-1 bucket, one launch instead of the chunk sum + the shard's AdamW pass: the reduced gradient of this rank's
// chunk (the chunk_sum_f32_kernel value, bitwise) is written into the fp32 gradient and applied to the shard's
// parameters / moments in the same pass, the updated bf16 parameters going straight into this rank's all-gather slot.
__global__ __launch_bounds__(256) void dp_sum_adamw_kernel(const bf16x4* __restrict__ in, int nchunks, size_t chunk4,
                                                           size_t n4, float4* __restrict__ grad, float4* __restrict__ p,
                                                           float4* __restrict__ m, float4* __restrict__ v,
                                                           bf16x4* __restrict__ shadow, AdamScalars sc) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) {
        float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int j = 0; j < nchunks; ++j) {
            const bf16x4 w = in[(size_t)j * chunk4 + i];
            s.x += bf2f(w[0]); s.y += bf2f(w[1]); s.z += bf2f(w[2]); s.w += bf2f(w[3]);
        }
        const float4 g = make_float4(bf2f(f2bf(s.x)), bf2f(f2bf(s.y)), bf2f(f2bf(s.z)), bf2f(f2bf(s.w)));
        grad[i] = g;
        float4 pp = nt_load4(p + i), mm = nt_load4(m + i), vv = nt_load4(v + i);
        bf16x4 o;
        adamw_one(pp, g, mm, vv, o, sc);
        nt_store4(p + i, pp);
        nt_store4(m + i, mm);
        nt_store4(v + i, vv);
        shadow[i] = o;
    }
}

// Pack a bucket for the all-to-all: dst[i] = bf16(src[i]) for i < n, 0 up to `total` (the padded W x chunk).
__global__ __launch_bounds__(256) void dp_pack_kernel(const float4* __restrict__ src, size_t n4, bf16x4* __restrict__ dst,
                                                      size_t total4) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < total4; i += (size_t)gridDim.x * 256) {
        bf16x4 o;
        if (i < n4) {
            const float4 x = src[i];
            o[0] = f2bf(x.x); o[1] = f2bf(x.y); o[2] = f2bf(x.z); o[3] = f2bf(x.w);
        } else {
            o[0] = o[1] = o[2] = o[3] = f2bf(0.f);
        }
        dst[i] = o;
    }
}

__global__ __launch_bounds__(256) void cast_f32_kernel(const bf16x4* __restrict__ src, float4* __restrict__ dst,
                                                       size_t n4) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) {
        const bf16x4 v = src[i];
        dst[i] = make_float4(bf2f(v[0]), bf2f(v[1]), bf2f(v[2]), bf2f(v[3]));
    }
}
}  // namespace ergm

extern "C" int ergm_chunk_sum_bf16(const void* in, int nchunks, size_t chunk, void* out, void* stream) {
    ERGM_CHECK_ARG(in && out && nchunks > 0 && chunk % 4 == 0, "chunk_sum_bf16: bad argument");
    const size_t c4 = chunk / 4;
    if (c4 == 0) return ERGM_OK;
    ERGM_LAUNCH(chunk_sum_kernel, dim3(grid_for(c4)), dim3(256), 0, as_stream(stream), (const bf16x4*)in,
                       nchunks, c4, (bf16x4*)out);
    return check_launch("chunk_sum_bf16");
}

extern "C" int ergm_chunk_sum_bf16_f32(const void* in, int nchunks, size_t chunk, size_t n, float* out, void* stream) {
    ERGM_CHECK_ARG(in && out && nchunks > 0 && chunk % 4 == 0 && n % 4 == 0 && n <= chunk,
                   "chunk_sum_bf16_f32: bad argument");
    const size_t n4 = n / 4;
    if (n4 == 0) return ERGM_OK;
    ERGM_LAUNCH(chunk_sum_f32_kernel, dim3(grid_for(n4)), dim3(256), 0, as_stream(stream), (const bf16x4*)in,
                       nchunks, chunk / 4, n4, (float4*)out);
    return check_launch("chunk_sum_bf16_f32");
}

extern "C" int ergm_cast_f32(const void* src, float* dst, size_t n, void* stream) {
    ERGM_CHECK_ARG(src && dst && n % 4 == 0, "cast_f32: bad argument");
    const size_t n4 = n / 4;
    if (n4 == 0) return ERGM_OK;
    ERGM_LAUNCH(cast_f32_kernel, dim3(grid_for(n4)), dim3(256), 0, as_stream(stream), (const bf16x4*)src,
                       (float4*)dst, n4);
    return check_launch("cast_f32");
}

extern "C" int ergm_dp_pack_bf16(const float* src, size_t n, void* dst, size_t total, void* stream) {
    ERGM_CHECK_ARG(src && dst && n % 4 == 0 && total % 4 == 0 && n <= total, "dp_pack_bf16: bad argument");
    ERGM_CHECK_ARG(aligned16(src) && (reinterpret_cast<uintptr_t>(dst) & 7) == 0, "dp_pack_bf16: alignment");
    const size_t t4 = total / 4;
    if (t4 == 0) return ERGM_OK;
    ERGM_LAUNCH(dp_pack_kernel, dim3(grid_for(t4)), dim3(256), 0, as_stream(stream), (const float4*)src, n / 4,
                (bf16x4*)dst, t4);
    return check_launch("dp_pack_bf16");
}

extern "C" int ergm_dp_sum_adamw(const void* in, int nchunks, size_t chunk, size_t n, float* grad, float* p, float* m,
                                 float* v, void* shadow, double lr, double beta1, double beta2, float eps,
                                 double weight_decay, float step_size, float bc2_sqrt, int max_blocks, void* stream) {
    ERGM_CHECK_ARG(in && grad && p && m && v && shadow && nchunks > 0 && chunk % 4 == 0 && n % 4 == 0 && n <= chunk,
                   "dp_sum_adamw: bad argument");
    ERGM_CHECK_ARG(max_blocks >= 0, "dp_sum_adamw: max_blocks must be >= 0");
    ERGM_CHECK_ARG(aligned16(grad) && aligned16(p) && aligned16(m) && aligned16(v) &&
                       (reinterpret_cast<uintptr_t>(shadow) & 7) == 0 && (reinterpret_cast<uintptr_t>(in) & 7) == 0,
                   "dp_sum_adamw: alignment");
    const size_t n4 = n / 4;
    if (n4 == 0) return ERGM_OK;
    const AdamScalars sc = adam_scalars(lr, beta1, beta2, eps, weight_decay, step_size, bc2_sqrt);
    unsigned grid = grid_for(n4);
    if (max_blocks > 0 && grid > (unsigned)max_blocks) grid = (unsigned)max_blocks;
    ERGM_LAUNCH(dp_sum_adamw_kernel, dim3(grid), dim3(256), 0, as_stream(stream), (const bf16x4*)in, nchunks,
                chunk / 4, n4, (float4*)grad, (float4*)p, (float4*)m, (float4*)v, (bf16x4*)shadow, sc);
    return check_launch("dp_sum_adamw");
}
