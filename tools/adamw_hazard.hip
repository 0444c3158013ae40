// AdamW hazard probe (gfx950): the production AdamW element pass (adamw.hip) against an exact host reference, alone and
// beside MFMA waves on the same CUs.  a replica probe (profiles/r06_adamw_replica_probe.txt) found replicas of the same update disagreeing in lanes 48-63
// (float4 components 0 / 2, mostly exp_avg_sq) when AdamW overlapped GEMMs; this isolates the kernel: the same inputs
// every iteration, outputs compared word for word with an IEEE float32 host computation (the kernel's arithmetic is all
// correctly rounded: no FMA contraction, IEEE sqrt and division).
// Variants: the production kernel (non-temporal, two float4 groups per thread) and rewrites of it; see kVariants.
// Usage: adamw_hazard <iters> [mfloats]
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../ergm_amd/csrc/common.h"

#define CK(x)                                                                               \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) {                                                             \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(2);                                                                        \
        }                                                                                   \
    } while (0)

using namespace ergm;

namespace ergm {
AdamScalars adam_scalars(double lr, double beta1, double beta2, float eps, double weight_decay, float step_size,
                         float bc2_sqrt) {
    return AdamScalars{(float)(1.0 - lr * weight_decay), (float)(1.0 - beta1), (float)beta2, (float)(1.0 - beta2), eps,
                       step_size, bc2_sqrt};
}
}  // namespace ergm

// ---- variant 0: the production kernel (adamw.hip adamw_kernel<true>) ----------------------------------------------
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
__device__ __forceinline__ float4 nt_load4(const float4* p) {
    f32x4 t = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p));
    return make_float4(t[0], t[1], t[2], t[3]);
}
__device__ __forceinline__ void nt_store4(float4* p, const float4& x) {
    __builtin_nontemporal_store(f32x4{x.x, x.y, x.z, x.w}, reinterpret_cast<f32x4*>(p));
}
__global__ __launch_bounds__(256) void v0_kernel(float4* __restrict__ p, const float4* __restrict__ g,
                                                 float4* __restrict__ m, float4* __restrict__ v,
                                                 bf16x4* __restrict__ pb, size_t n4, AdamScalars sc) {
    const size_t stride = (size_t)gridDim.x * 256;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += 2 * stride) {
        const size_t i2 = i + stride;
        const bool two = i2 < n4;
        float4 p0 = nt_load4(p + i), g0 = nt_load4(g + i), m0 = nt_load4(m + i), v0 = nt_load4(v + i);
        float4 p1, g1, m1, v1;
        if (two) {
            p1 = nt_load4(p + i2);
            g1 = nt_load4(g + i2);
            m1 = nt_load4(m + i2);
            v1 = nt_load4(v + i2);
        }
        bf16x4 o0, o1;
        adamw_one(p0, g0, m0, v0, o0, sc);
        nt_store4(p + i, p0);
        nt_store4(m + i, m0);
        nt_store4(v + i, v0);
        if (pb) pb[i] = o0;
        if (two) {
            adamw_one(p1, g1, m1, v1, o1, sc);
            nt_store4(p + i2, p1);
            nt_store4(m + i2, m1);
            nt_store4(v + i2, v1);
            if (pb) pb[i2] = o1;
        }
    }
}

// ---- variant 1: one element per lane (scalar loads, no packed-math pairing possible across components) --------------
__global__ __launch_bounds__(256) void v1_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                                                 float* __restrict__ v, __bf16* __restrict__ pb, size_t n, AdamScalars sc) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        float mm = m[i], vv = v[i];
        const float x = adamw_elem(p[i], g[i], mm, vv, sc);
        p[i] = x;
        m[i] = mm;
        v[i] = vv;
        if (pb) pb[i] = f2bf(x);
    }
}

// ---- variant 2: the smallest form, a chain of fused multiply-adds on float pairs (v_pk_fma_f32 when packed FP32
// instructions are enabled, two v_fma_f32 otherwise) -------------------------------------------------------------------
__global__ __launch_bounds__(256) void v2_kernel(float2* __restrict__ x, size_t n2, int chain, float c, float d) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n2; i += (size_t)gridDim.x * 256) {
        float2 v = x[i];
        for (int k = 0; k < chain; ++k) {
            v.x = __builtin_fmaf(v.x, c, d);
            v.y = __builtin_fmaf(v.y, c, d);
        }
        x[i] = v;
    }
}

// ---- MFMA pressure: waves that keep the matrix cores busy on every SIMD while AdamW runs ------------------------------
__global__ __launch_bounds__(256) void mfma_spin(float* out, int iters) {
    bf16x8 a, b;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        a[j] = (__bf16)(0.001f * (threadIdx.x + j));
        b[j] = (__bf16)(0.002f * (j + 1));
    }
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < iters; ++k) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
    if (acc[0] == -1.f) out[threadIdx.x] = acc[1];
}

// ---- compare device result with the host reference, log the first mismatches (offset, component, lane) ----------------
__global__ __launch_bounds__(256) void compare(const float* got, const float* want, size_t n, unsigned* bad, unsigned* log) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        if (__float_as_uint(got[i]) != __float_as_uint(want[i])) {
            const unsigned k = atomicAdd(bad, 1u);
            if (k < 32) log[k] = (unsigned)i;
        }
    }
}

static float host_elem(float p, float g, float& m, float& v, const AdamScalars& s) {
    volatile float x = p * s.decay;
    volatile float d = g - m;
    volatile float t = s.one_m_b1 * d;
    const float mj = m + t;
    volatile float gg = g * g;
    volatile float a = v * s.b2;
    volatile float b = s.one_m_b2 * gg;
    const float vj = a + b;
    volatile float sq = std::sqrt(vj);
    volatile float den0 = sq / s.bc2_sqrt;
    const float denom = den0 + s.eps;
    volatile float q = mj / denom;
    volatile float u = (-s.step_size) * q;
    m = mj;
    v = vj;
    return x + u;
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 200;
    const size_t n = (size_t)(argc > 2 ? atoi(argv[2]) : 4) << 20;
    std::vector<float> hp(n), hg(n), hm(n), hv(n);
    unsigned s = 12345;
    auto rnd = [&]() { s = s * 1664525u + 1013904223u; return ((s >> 8) * (1.0f / 16777216.0f)) - 0.5f; };
    for (size_t i = 0; i < n; ++i) {
        hp[i] = 0.04f * rnd();
        hg[i] = 0.002f * rnd();
        hm[i] = 0.001f * rnd();
        hv[i] = 1e-6f * (rnd() + 0.5f);
    }
    const double lr = 5.8e-4, b1 = 0.9, b2 = 0.999, wd = 0.01;
    const int t = 12;
    const AdamScalars sc = adam_scalars(lr, b1, b2, 1e-8f, wd, (float)(lr / (1 - std::pow(b1, t))),
                                        (float)std::sqrt(1 - std::pow(b2, t)));
    std::vector<float> rp(n), rm(hm), rv(hv);
    for (size_t i = 0; i < n; ++i) rp[i] = host_elem(hp[i], hg[i], rm[i], rv[i], sc);
    float *p, *g, *m, *v, *p0, *m0, *v0, *wp, *wm, *wv, *sink;
    __bf16* pb;
    unsigned *bad, *log;
    const size_t B = n * 4;
    for (float** q : {&p, &g, &m, &v, &p0, &m0, &v0, &wp, &wm, &wv}) CK(hipMalloc(q, B));
    CK(hipMalloc(&pb, n * 2));
    CK(hipMalloc(&sink, 4096));
    CK(hipMalloc(&bad, 16));
    CK(hipMalloc(&log, 3 * 32 * 4));
    CK(hipMemcpy(p0, hp.data(), B, hipMemcpyHostToDevice));
    CK(hipMemcpy(g, hg.data(), B, hipMemcpyHostToDevice));
    CK(hipMemcpy(m0, hm.data(), B, hipMemcpyHostToDevice));
    CK(hipMemcpy(v0, hv.data(), B, hipMemcpyHostToDevice));
    CK(hipMemcpy(wp, rp.data(), B, hipMemcpyHostToDevice));
    CK(hipMemcpy(wm, rm.data(), B, hipMemcpyHostToDevice));
    CK(hipMemcpy(wv, rv.data(), B, hipMemcpyHostToDevice));
    hipStream_t s1, s2;
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    const size_t BK = 232704;  // the trainer test's bucket: 114 workgroups of the production grid
    {  // variant 2: fma chains on float pairs
        const int chain = 64;
        const float c = 0.999f, d = 1e-4f;
        std::vector<float> rx(hp);
        for (size_t i = 0; i < n; ++i)
            for (int k = 0; k < chain; ++k) rx[i] = std::fma(rx[i], c, d);
        CK(hipMemcpy(wp, rx.data(), B, hipMemcpyHostToDevice));
        for (int pressure = 0; pressure < 2; ++pressure) {
            unsigned tot = 0, first[32];
            bool have = false;
            for (int it = 0; it < iters; ++it) {
                CK(hipMemcpyAsync(p, p0, B, hipMemcpyDeviceToDevice, s1));
                CK(hipMemsetAsync(bad, 0, 16, s1));
                CK(hipStreamSynchronize(s1));
                if (pressure) hipLaunchKernelGGL(mfma_spin, dim3(1024), dim3(256), 0, s2, sink, 20000);
                hipLaunchKernelGGL(v2_kernel, dim3(2048), dim3(256), 0, s1, (float2*)p, n / 2, chain, c, d);
                hipLaunchKernelGGL(compare, dim3(2048), dim3(256), 0, s1, p, wp, n, bad, log);
                CK(hipStreamSynchronize(s1));
                CK(hipStreamSynchronize(s2));
                unsigned nb[4], lg[32];
                CK(hipMemcpy(nb, bad, 16, hipMemcpyDeviceToHost));
                CK(hipMemcpy(lg, log, sizeof(lg), hipMemcpyDeviceToHost));
                tot += nb[0];
                if (nb[0] && !have) {
                    have = true;
                    memcpy(first, lg, sizeof(lg));
                }
            }
            printf("variant 2 (fma chain on float pairs) %s: wrong words %u over %d iterations of %zu M\n",
                   pressure ? "beside MFMA waves" : "alone", tot, iters, n >> 20);
            if (have) {
                printf("   first:");
                for (int k = 0; k < 8; ++k)
                    printf(" %u(comp %u of pair, lane %u)", first[k], first[k] % 2, (unsigned)(first[k] / 2 % 64));
                printf("\n");
            }
            fflush(stdout);
        }
        CK(hipMemcpy(wp, rp.data(), B, hipMemcpyHostToDevice));
    }
    for (int variant = 0; variant < 2; ++variant) {
        for (int pressure = 0; pressure < 2; ++pressure) {
            unsigned tot[3] = {0, 0, 0};
            unsigned first[3][32];
            bool have[3] = {false, false, false};
            for (int it = 0; it < iters; ++it) {
                CK(hipMemcpyAsync(p, p0, B, hipMemcpyDeviceToDevice, s1));
                CK(hipMemcpyAsync(m, m0, B, hipMemcpyDeviceToDevice, s1));
                CK(hipMemcpyAsync(v, v0, B, hipMemcpyDeviceToDevice, s1));
                CK(hipMemsetAsync(bad, 0, 16, s1));
                CK(hipStreamSynchronize(s1));
                if (pressure) hipLaunchKernelGGL(mfma_spin, dim3(1024), dim3(256), 0, s2, sink, 20000);
                for (size_t a = 0; a < n; a += BK) {
                    const size_t len = std::min(BK, n - a);
                    if (variant == 0) {
                        const size_t n4 = len / 4;
                        unsigned grid = (unsigned)std::min<size_t>((n4 + 511) / 512, 4096);
                        hipLaunchKernelGGL(v0_kernel, dim3(grid), dim3(256), 0, s1, (float4*)(p + a), (const float4*)(g + a),
                                           (float4*)(m + a), (float4*)(v + a), (bf16x4*)(pb + a), n4, sc);
                    } else {
                        unsigned grid = (unsigned)std::min<size_t>((len + 255) / 256, 8192);
                        hipLaunchKernelGGL(v1_kernel, dim3(grid), dim3(256), 0, s1, p + a, g + a, m + a, v + a, pb + a, len,
                                           sc);
                    }
                }
                const float* got[3] = {p, m, v};
                const float* want[3] = {wp, wm, wv};
                for (int b = 0; b < 3; ++b)
                    hipLaunchKernelGGL(compare, dim3(2048), dim3(256), 0, s1, got[b], want[b], n, bad + b, log + 32 * b);
                CK(hipStreamSynchronize(s1));
                CK(hipStreamSynchronize(s2));
                unsigned nb[4], lg[96];
                CK(hipMemcpy(nb, bad, 16, hipMemcpyDeviceToHost));
                CK(hipMemcpy(lg, log, sizeof(lg), hipMemcpyDeviceToHost));
                for (int b = 0; b < 3; ++b) {
                    tot[b] += nb[b];
                    if (nb[b] && !have[b]) {
                        have[b] = true;
                        memcpy(first[b], lg + 32 * b, 32 * 4);
                    }
                }
            }
            printf("variant %d (%s) %s: wrong words param %u exp_avg %u exp_avg_sq %u over %d iterations of %zu M\n",
                   variant, variant == 0 ? "production float4 x2, nt" : "one element per lane",
                   pressure ? "beside MFMA waves" : "alone", tot[0], tot[1], tot[2], iters, n >> 20);
            for (int b = 0; b < 3; ++b)
                if (have[b]) {
                    printf("   buffer %d first:", b);
                    for (int k = 0; k < 8; ++k) {
                        const unsigned o = first[b][k];
                        printf(" %u(mod256 %u, comp %u, lane %u)", o, o % 256, o % 4, (unsigned)((o % BK) / 4 % 64));
                    }
                    printf("\n");
                }
            fflush(stdout);
        }
    }
    return 0;
}
